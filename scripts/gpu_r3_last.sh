#!/bin/bash
# Last call of the session: AdamW kernel tests (modes 0/1/2), Llama-3 8B A/B of the plain-load 8-wide AdamW, then a
# rocprofv3 kernel trace of the final ResNet-50 Hyperband bench (summary under gpurun_out/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_lm.py -k "adamw or optimizer_in_backward" > gpurun_out/last_tests.log 2>&1
rc=$?; tail -2 gpurun_out/last_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in PLX_ADAMW_WIDE=2 PLX_ADAMW_WIDE=0 PLX_ADAMW_WIDE=2 PLX_ADAMW_WIDE=0; do
  i=$((i + 1))
  env $v timeout -k 10 400 python scripts/bench_suite.py --only lm_llama8b --quick > gpurun_out/last_llama_$i.jsonl 2> gpurun_out/last_llama_$i.err || { echo "variant '$v' failed"; tail -5 gpurun_out/last_llama_$i.err; exit 1; }
  echo "llama [$v] $(python -c "import json; d=json.loads(open('gpurun_out/last_llama_$i.jsonl').read().strip().splitlines()[-1]); print(d['tokens_per_s'])")"
done
PROF_TAG=r3_final_prefetch bash scripts/prof_only.sh
