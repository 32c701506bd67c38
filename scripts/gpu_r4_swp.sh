#!/bin/bash
# Round 4: software-pipelined NT conv kernels (PLX_SWP) -- numerics, isolated A/B on the 3x3 shapes, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "software_pipelined" \
  > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
timeout -k 10 300 python scripts/conv_ab.py ti,swp4,swp5 5 fwd,dgrad > gpurun_out/r4s_ab.jsonl 2> gpurun_out/r4s_ab.err \
  || { tail -20 gpurun_out/r4s_ab.err; exit 1; }
cat gpurun_out/r4s_ab.jsonl | cut -c1-400
if [ -n "${AB_LIST:-}" ]; then
  TAG=r4s_bench bash scripts/gpu_ab_multi.sh || exit 1
fi
