#!/bin/bash
# rocprofv3 kernel trace of a short bench run (build first), for scripts/prof_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/pbuild.log 2>&1 \
&& timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
