#!/bin/bash
# Stream priorities: GPU test, then bench A/B (main stream high / side stream low / both)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_priority.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4prio_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4prio_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_LIST="PLX_MAIN_PRIORITY=-1;;PLX_WGRAD_PRIORITY=1;PLX_MAIN_PRIORITY=-1 PLX_WGRAD_PRIORITY=1;PLX_MAIN_PRIORITY=-1;PLX_MAIN_PRIORITY=0" TAG=r4prio bash scripts/gpu_ab_multi.sh
