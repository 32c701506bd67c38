#!/bin/bash
# Round 4: the RCCL fix (GPU_MAX_HW_QUEUES=8 by default) -- communicator early vs after the timed region, and the
# Llama-3 8B world-1 all-reduce path, all at the new default
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import os, polyaxon_amd; print('GPU_MAX_HW_QUEUES', os.environ['GPU_MAX_HW_QUEUES'])"
AB_LIST="PLX_BENCH_RCCL=early;;PLX_BENCH_RCCL=early;" TAG=r4fix bash scripts/gpu_ab_multi.sh || exit 1
T="python -m polyaxon_amd.trainers lm --model llama3_8b --bs 1 --seq 4096 --steps 20 --lr 3e-4 --log_every 5"
for v in "" "--world1_collectives all" "--world1_collectives metric" ""; do
  timeout -k 10 400 $T $v > gpurun_out/r4fix_c5.log 2>&1 || { tail -20 gpurun_out/r4fix_c5.log; exit 1; }
  echo "llama [$v] $(grep '^{' gpurun_out/r4fix_c5.log | tail -1 | cut -c1-200)"
done
