#!/bin/bash
# GPT-2 trainer, 40 steps: no collectives / world-1 collectives with planned buckets / with 64 MB buckets
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for args in "" "--world1_collectives all" "--world1_collectives all --bucket_mb 64" ""; do
  i=$((i + 1))
  timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 40 $args > gpurun_out/r4bk_$i.json 2> gpurun_out/r4bk_$i.err || { tail -20 gpurun_out/r4bk_$i.err; exit 1; }
  echo "[$args] $(python -c "import json; d=json.loads(open('gpurun_out/r4bk_$i.json').read().strip().splitlines()[-1]); print(d['tokens_per_s'], d['buckets'], d['bucket_launches'])")"
done
