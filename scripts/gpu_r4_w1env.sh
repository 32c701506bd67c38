#!/bin/bash
# GPT-2 world-1 bucket all-reduces through ProcessGroupNCCL: which torch/RCCL setting makes the host stall?
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for envs in "" "TORCH_NCCL_AVOID_RECORD_STREAMS=1" "TORCH_NCCL_ASYNC_ERROR_HANDLING=0" "TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_AVOID_RECORD_STREAMS=1" "TORCH_NCCL_ENABLE_TIMING=0 TORCH_NCCL_TRACE_BUFFER_SIZE=0" "NCCL_LAUNCH_MODE=GROUP"; do
  i=$((i + 1))
  env $envs timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 40 --world1_collectives all > gpurun_out/r4env_$i.json 2> gpurun_out/r4env_$i.err || { tail -20 gpurun_out/r4env_$i.err; exit 1; }
  echo "[$envs] $(python -c "import json; d=json.loads(open('gpurun_out/r4env_$i.json').read().strip().splitlines()[-1]); print(d['tokens_per_s'])")"
done
