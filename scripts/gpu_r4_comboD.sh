#!/bin/bash
# Round 4: config 4 process mode at the resident bench's 40 steps per trial, then config 5 (Llama-3 8B, DP=1):
# bare trainer vs --world1_collectives vs --zero1, and the same job through plx run
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/gpt2_bo_process.py --steps 40 > gpurun_out/r4_gpt2_bo_process_40steps.json \
  2> gpurun_out/r4_gpt2_bo_process_40steps.err || { tail -30 gpurun_out/r4_gpt2_bo_process_40steps.err; exit 1; }
cat gpurun_out/r4_gpt2_bo_process_40steps.json
bash scripts/gpu_r4_config5.sh || exit 1
