#!/bin/bash
# Wide weight-gradient tiles: numerics (new + existing TN tests), the round-end tiers (pytest -m gpu, smoke), then an
# interleaved A/B of PLX_TN_WIDE on the default bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "tn_wide or stage_rings" > gpurun_out/wide_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wide_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=wide AB_LIST="${AB_LIST:-PLX_TN_WIDE=0;PLX_TN_WIDE=1;PLX_TN_WIDE=0;PLX_TN_WIDE=1}" bash scripts/gpu_ab_multi.sh
