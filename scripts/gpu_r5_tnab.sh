#!/bin/bash
# ResNet-50 bench A/B, alternating: weight-gradient kernel v1 (gemm_tn_kernel) vs v2 (wgrad_kernel).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r5tn}.jsonl
: > $OUT
STEPS=${STEPS:-3}
for v in ${VARIANTS:-0 1,64 0 1,64}; do
  PLX_TN_V2="$v" timeout -k 10 420 python -u bench.py --steps $STEPS --warmup 1 > gpurun_out/_tn.json 2> gpurun_out/${TAG:-r5tn}_${v/,/_}.err || { tail -5 gpurun_out/${TAG:-r5tn}_${v/,/_}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/_tn.json').read().strip().splitlines()[-1]); print(json.dumps({'tn_v2': '$v', 'value': d['value'], 'train_images_per_s': d['train_images_per_s'], 'ms_per_step': d['ms_per_step']}))" >> $OUT
  tail -1 $OUT
done
