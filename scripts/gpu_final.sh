#!/bin/bash
# Round-end rehearsal of the driver's GPU tiers on the in-tree .so files (no rebuild): full pytest -m gpu, smoke(),
# then the default bench; each GPU step under its own time limit, stopping at the first failure
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
rc=$?; cut -c1-600 gpurun_out/final_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/final_bench.err; exit $rc; }
exit 0
