#!/bin/bash
# LM iteration: LM / attention GPU tests, then tokens/s for the default path and an A/B variant (AB="ENV=VAL")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-lmit}
timeout -k 10 400 python -u -m pytest tests/test_gpu_lm.py tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_test.log; [ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/${TAG}_test.log | head -20; exit $rc; }
TAG=${TAG} bash scripts/gpu_lm_tokens.sh || exit 1
if [ -n "${AB:-}" ]; then env $AB bash -c "TAG=${TAG}_ab bash scripts/gpu_lm_tokens.sh" || exit 1; fi
