#!/bin/bash
# Round 4: 4-wave GEMM tests + bench, then the 10-sweep Hyperband / ASHA benches (one box acquisition)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r4_gemm.sh || exit 1
bash scripts/gpu_r4_sweeps.sh || exit 1
