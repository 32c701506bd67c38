#!/bin/bash
# Round 4: why a live RCCL communicator slows the ResNet-50 bench (verdict r3 weak #3).  Alternating 3-sweep bench
# runs with the communicator created before the warm-up (PLX_BENCH_RCCL=early) or after the timed region (default),
# then with more HIP hardware queues, then a kernel trace of the early-communicator run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_LIST="${AB_LIST:-PLX_BENCH_RCCL=early;;PLX_BENCH_RCCL=early GPU_MAX_HW_QUEUES=8;GPU_MAX_HW_QUEUES=8;PLX_BENCH_RCCL=early}" \
  TAG=r4rccl bash scripts/gpu_ab_multi.sh || exit 1
if [ "${LLAMA:-1}" = "1" ]; then  # bucket size vs the per-collective cost of the world-1 all-reduce path
  T="python -m polyaxon_amd.trainers lm --model llama3_8b --bs 1 --seq 4096 --steps 20 --lr 3e-4 --log_every 5"
  for v in "--world1_collectives all --bucket_mb 512" "--world1_collectives all --bucket_mb 2048" "--bucket_mb 512"; do
    timeout -k 10 400 $T $v > gpurun_out/r4rccl_c5.log 2>&1 || { tail -20 gpurun_out/r4rccl_c5.log; exit 1; }
    echo "llama [$v] $(grep '^{' gpurun_out/r4rccl_c5.log | tail -1 | cut -c1-200)"
  done
fi
if [ "${PROF:-1}" = "1" ]; then
  PROF_TAG=r4rccl_base_resnet50_hb STEPS=2 bash scripts/prof_only.sh || exit 1
  PLX_BENCH_RCCL=early PROF_TAG=r4rccl_early_resnet50_hb STEPS=2 bash scripts/prof_only.sh || exit 1
  head -16 gpurun_out/r4rccl_base_resnet50_hb_steady_state.md
  head -16 gpurun_out/r4rccl_early_resnet50_hb_steady_state.md
  python scripts/kernel_stats_diff.py gpurun_out/r4rccl_base_resnet50_hb_kernel_stats.csv \
    gpurun_out/r4rccl_early_resnet50_hb_kernel_stats.csv > gpurun_out/r4rccl_kernel_diff.md
  head -30 gpurun_out/r4rccl_kernel_diff.md
fi
