#!/bin/bash
# Round 4 end-of-session check: the GPU test suite, smoke(), and the driver-shaped bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4final_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4final_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final_smoke.log 2>&1 || { tail -20 gpurun_out/r4final_smoke.log; exit 1; }
tail -2 gpurun_out/r4final_smoke.log
