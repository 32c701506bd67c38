#!/bin/bash
# round-3 first probe: GP Cholesky race-fix tests + list of PMC counters available on the box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1
echo "list-avail rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_gp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gp_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gp_tests.log
echo "exit $rc"
exit $rc
