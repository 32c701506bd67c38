#!/bin/bash
# ResNet path iteration: conv / BN numerics tests, then a short bench (each GPU step under its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-bn}
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; cut -c1-400 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
if [ -n "${AB:-}" ]; then  # A/B: the same bench with an env knob flipped (e.g. AB="PLX_BN_SUMS=0")
  env $AB timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_ab.json 2> gpurun_out/${TAG}_bench_ab.err || exit 1
  echo "A/B ($AB):"; cut -c1-300 gpurun_out/${TAG}_bench_ab.json
fi
[ -n "${LM:-}" ] && TAG=${TAG}_lm bash scripts/gpu_lm_tokens.sh
exit 0
