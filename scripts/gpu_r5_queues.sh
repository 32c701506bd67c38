#!/bin/bash
# Hardware-queue A/B of the ResNet-50 bench with a live RCCL communicator (PLX_BENCH_RCCL=early, the default):
# the box's own GPU_MAX_HW_QUEUES vs 8 queues, and the weight-gradient side stream's priority level.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r5q}.jsonl
: > $OUT
STEPS=${STEPS:-3}
run() {  # name, env assignments...
  local name=$1; shift
  echo "== $name (GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset} $*)" >&2
  env "$@" timeout -k 10 420 python -u bench.py --steps $STEPS --warmup 1 > gpurun_out/_q.json 2> gpurun_out/${TAG:-r5q}_$name.err || { echo "$name failed" >&2; tail -5 gpurun_out/${TAG:-r5q}_$name.err >&2; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/_q.json').read().strip().splitlines()[-1]); print(json.dumps({'variant': '$name', 'value': d['value'], 'train_images_per_s': d['train_images_per_s'], 'ms_per_step': d['ms_per_step'], 'control': d.get('control_device_footprint')}))" >> $OUT
  tail -1 $OUT >&2
}
for v in ${VARIANTS:-q4 q4_hi q4_lo q8 q4}; do
  case $v in
    q4) run q4 PLX_WGRAD_PRIORITY= || exit 1 ;;
    q4_hi) run q4_hi PLX_WGRAD_PRIORITY=-1 || exit 1 ;;
    q4_lo) run q4_lo PLX_WGRAD_PRIORITY=1 || exit 1 ;;
    q8) run q8 PLX_HW_QUEUES=8 PLX_WGRAD_PRIORITY= || exit 1 ;;
  esac
done
cat $OUT
