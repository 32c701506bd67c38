#!/bin/bash
# attention iteration: numerics tests, microbenchmark, per-kernel profile (each step under its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-attn}
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_test.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG} bash scripts/gpu_attn.sh || exit $?
TAG=${TAG}_prof bash scripts/gpu_attn_prof.sh
