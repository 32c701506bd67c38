#!/bin/bash
# GPU box: the non-headline BASELINE configs (scripts/bench_suite.py) + the GP kernel tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gp.log 2>&1 \
&& timeout -k 10 900 python scripts/bench_suite.py --only ${SUITE:-iris,hb_reduce,bo,mlp_grid,lm_gpt2,lm_llama8b} --bo-backends hip ${SUITE_ARGS:-} > gpurun_out/suite.jsonl 2> gpurun_out/suite.err
rc=$?
tail -3 gpurun_out/pytest_gp.log
cat gpurun_out/suite.jsonl
echo "exit $rc"
exit $rc
