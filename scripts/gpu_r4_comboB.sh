#!/bin/bash
# Round 4: 4-wave GEMM (tests + bench) then the software-pipelined conv kernels (tests, isolated A/B, bench A/B)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r4_gemm.sh || exit 1
AB_LIST="${AB_LIST-PLX_SWP=4,0;}" bash scripts/gpu_r4_swp.sh || exit 1
