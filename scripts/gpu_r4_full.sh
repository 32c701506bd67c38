#!/bin/bash
# round 4: GPU test suite, bench A/B (AB_LIST), rocprofv3 steady-state profile of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4full}
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${AB_LIST:-}" ]; then
  TAG=${TAG}_ab bash scripts/gpu_ab_multi.sh || exit 1
fi
if [ "${PROF:-1}" = "1" ]; then
  PROF_TAG=${TAG}_resnet50_hb STEPS=2 bash scripts/prof_only.sh || exit 1
  head -14 gpurun_out/${TAG}_resnet50_hb_steady_state.md
fi
