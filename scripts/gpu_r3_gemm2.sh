#!/bin/bash
# round 3: LM GEMM kernel (5-deep DMA ring) numerics + speed vs hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_pytest.log 2>&1 \
&& echo "gemm tests ok" \
&& timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench2.jsonl 2> gpurun_out/gemm_bench2.err \
&& echo "gemm bench ok" \
&& PLX_GEMM_SPLIT_TARGET=0 timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench2_nosplit.jsonl 2> gpurun_out/gemm_bench2_nosplit.err
rc=$?
echo "exit $rc"
tail -3 gpurun_out/gemm_pytest.log
exit $rc
