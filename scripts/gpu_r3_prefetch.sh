#!/bin/bash
# Side-stream batch prefetch: GPU test vs inline generation, then an interleaved A/B of PLX_PREFETCH_BATCH
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_synth.py > gpurun_out/prefetch_tests.log 2>&1
rc=$?; tail -2 gpurun_out/prefetch_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=prefetch AB_LIST="${AB_LIST:-PLX_PREFETCH_BATCH=0;PLX_PREFETCH_BATCH=1;PLX_PREFETCH_BATCH=0;PLX_PREFETCH_BATCH=1}" bash scripts/gpu_ab_multi.sh
