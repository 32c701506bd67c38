#!/bin/bash
# GPU box: conv/BN/kernel tests, eager and hipGraph bench, kernel-trace profile of the chosen mode.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bn.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fusion.log 2>&1 \
&& timeout -k 10 600 python bench.py --steps 13 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json \
&& timeout -k 10 600 python bench.py --steps 13 --warmup 2 --graph > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err && cat gpurun_out/bench_graph.json \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_fusion.log
echo "exit $rc"
exit $rc
