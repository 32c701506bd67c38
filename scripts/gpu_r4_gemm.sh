#!/bin/bash
# Round 4: the 4-wave AGPR GEMM kernel -- numerics tests, then the in-process 8-wave / 4-wave / hipBLASLt bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_models.py \
  > gpurun_out/r4g_tests.log 2>&1 || { tail -40 gpurun_out/r4g_tests.log; exit 1; }
tail -3 gpurun_out/r4g_tests.log
timeout -k 10 400 python scripts/gemm_bench.py --waves ${WAVES:-8,4,5,6,7} > gpurun_out/r4g_bench.jsonl 2> gpurun_out/r4g_bench.err \
  || { tail -20 gpurun_out/r4g_bench.err; exit 1; }
cat gpurun_out/r4g_bench.jsonl
