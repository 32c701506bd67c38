#!/bin/bash
# round 3: LM GEMM kernel numerics + speed vs hipBLASLt, then the 1-GPU bench (halo now off by default)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_pytest.log 2>&1 \
&& echo "gemm tests ok" \
&& timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err \
&& echo "gemm bench ok" \
&& timeout -k 10 400 python bench.py --steps 3 --warmup 1 --target 0.02 > gpurun_out/bench_r3g.json 2> gpurun_out/bench_r3g.err \
&& cat gpurun_out/bench_r3g.json | cut -c1-300
rc=$?
echo "exit $rc"
tail -3 gpurun_out/gemm_pytest.log
exit $rc
