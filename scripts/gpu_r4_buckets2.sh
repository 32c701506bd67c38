#!/bin/bash
# GPT-2 trainer, 40 steps, world-1 collectives: is the cost the hardware-queue count again?
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in ":" "PLX_HW_QUEUES=16:--world1_collectives all" ":--world1_collectives all" "PLX_HW_QUEUES=16:" ":--world1_collectives metric" "PLX_HW_QUEUES=32:--world1_collectives all"; do
  i=$((i + 1))
  envs=${v%%:*}; args=${v#*:}
  env $envs timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 40 $args > gpurun_out/r4bq_$i.json 2> gpurun_out/r4bq_$i.err || { tail -20 gpurun_out/r4bq_$i.err; exit 1; }
  echo "[$envs $args] $(python -c "import json; d=json.loads(open('gpurun_out/r4bq_$i.json').read().strip().splitlines()[-1]); print(d['tokens_per_s'], d['buckets'], d['bucket_launches'])")"
done
