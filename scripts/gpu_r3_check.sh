#!/bin/bash
# round-3 GPU check: gpu tests, hyperband + asha benches (each GPU step under its own limit; stop at first failure)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-3}
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& tail -2 gpurun_out/pytest_gpu.log \
&& echo "== bench hyperband" && timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench_hb.json 2> gpurun_out/bench_hb.err \
&& cat gpurun_out/bench_hb.json \
&& echo "== bench asha" && timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 --search asha ${BENCH_ARGS:-} > gpurun_out/bench_asha.json 2> gpurun_out/bench_asha.err \
&& cat gpurun_out/bench_asha.json
rc=$?
tail -3 gpurun_out/pytest_gpu.log
echo "exit $rc"
exit $rc
