#!/bin/bash
# One on-box iteration: build, the GPU tests in $TESTS, a short bench and a rocprofv3 kernel trace of it
# summarised on the box (PROF_TAG names the files).  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${PROF_TAG:-iter}
TESTS=${TESTS:-tests/test_gpu_conv.py}
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/ibuild.log 2>&1 \
&& timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 \
&& timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
&& cat gpurun_out/${TAG}_bench.json \
&& timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/plx_prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
trace=$(ls /tmp/plx_prof/*/run_kernel_trace.csv /tmp/plx_prof/run_kernel_trace.csv 2>/dev/null | head -1)
if [ $rc -eq 0 ] && [ -n "$trace" ]; then
  python scripts/prof_summary.py "$trace" --steps 40 --top 40 --markdown > gpurun_out/${TAG}_steady_state.md
fi
echo "exit $rc"
exit $rc
