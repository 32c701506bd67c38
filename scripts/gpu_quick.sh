#!/bin/bash
# build + full GPU test suite + a 3-sweep bench (no profile); each GPU step under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/qbuild.log 2>&1 \
&& timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& cat gpurun_out/bench.json
rc=$?
tail -2 gpurun_out/pytest_gpu.log
echo "exit $rc"
exit $rc
