#!/bin/bash
# rocprofv3 kernel trace of a short bench run (build first), summarised on the box by scripts/prof_summary.py
# (the raw trace is larger than gpurun copies back); PROF_TAG names the summary files
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${PROF_TAG:-prof}
rm -rf /tmp/plx_prof  # one trace per run: the summary below picks the first trace directory it finds
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/pbuild.log 2>&1 \
&& timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/plx_prof -o run --output-format csv -- python bench.py --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/$TAG.log 2>&1
rc=$?
trace=$(ls /tmp/plx_prof/*/run_kernel_trace.csv /tmp/plx_prof/run_kernel_trace.csv 2>/dev/null | head -1)
if [ $rc -eq 0 ] && [ -n "$trace" ]; then
  python scripts/prof_summary.py "$trace" --steps 40 --top 40 --markdown > gpurun_out/${TAG}_steady_state.md
  stats=$(ls /tmp/plx_prof/*/run_kernel_stats.csv /tmp/plx_prof/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$stats" ] && cp "$stats" gpurun_out/${TAG}_kernel_stats.csv
fi
echo "exit $rc"
exit $rc
