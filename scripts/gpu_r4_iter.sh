#!/bin/bash
# Round 4 kernel iteration: selected GPU tests, then the conv A/B (scripts/conv_ab.py).
#   TESTS="tests/test_gpu_conv.py -k ring" VARIANTS=base,v2 scripts/gpu_r4_iter.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4it}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -25 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${VARIANTS:-}" ]; then
  timeout -k 10 400 python -u scripts/conv_ab.py "$VARIANTS" "${ROUNDS:-7}" "${PASSES:-fwd,dgrad}" "${SHAPES:-all}" \
    > gpurun_out/${TAG}_ab.jsonl 2> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
  cat gpurun_out/${TAG}_ab.jsonl
fi
