#!/bin/bash
# GPT-2 world-1 bucket all-reduces: RCCL AVG (pre-multiplied sum) vs SUM + 1/W scale
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in ":--world1_collectives all" "PLX_DDP_AVG=0:--world1_collectives all" ":" "PLX_DDP_AVG=0:--world1_collectives all --zero1" ":--world1_collectives all --zero1"; do
  i=$((i + 1))
  envs=${v%%:*}; args=${v#*:}
  env $envs timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 40 $args > gpurun_out/r4avg_$i.json 2> gpurun_out/r4avg_$i.err || { tail -20 gpurun_out/r4avg_$i.err; exit 1; }
  echo "[$envs $args] $(python -c "import json; d=json.loads(open('gpurun_out/r4avg_$i.json').read().strip().splitlines()[-1]); print(d['tokens_per_s'], d['loss'], d['buckets'], d['bucket_launches'])")"
done
