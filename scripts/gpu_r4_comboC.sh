#!/bin/bash
# Round 4: config 4 (resident BO bench + the same group in process mode), then the 10-sweep Hyperband / ASHA benches
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
(rocm-smi --showclocks --showpower --showuse 2>&1 | head -40) > gpurun_out/r4c_box.txt || true
BO=1 BOP=1 C5=0 RCCL=0 bash scripts/gpu_r4_multi.sh || exit 1
bash scripts/gpu_r4_sweeps.sh || exit 1
