#!/bin/bash
# LM A/B on one box: 8-wide non-temporal AdamW (PLX_ADAMW_WIDE) and the fused residual add + RMSNorm (PLX_ADD_LN),
# after the optimizer kernel tests; each run under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_lm.py -k "adamw or optimizer_in_backward" > gpurun_out/lmab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lmab_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra VARIANTS <<< "${AB_LIST:-PLX_ADAMW_WIDE=1;PLX_ADAMW_WIDE=0;PLX_ADD_LN=0;PLX_ADAMW_WIDE=1;PLX_ADAMW_WIDE=0;PLX_ADD_LN=0}"
for v in "${VARIANTS[@]}"; do
  i=$((i + 1))
  env $v timeout -k 10 400 python scripts/bench_suite.py --only lm_llama8b --quick > gpurun_out/lmab_llama_$i.jsonl 2> gpurun_out/lmab_llama_$i.err || { echo "variant '$v' failed"; tail -5 gpurun_out/lmab_llama_$i.err; exit 1; }
  echo "llama [$v] $(python -c "import json; d=json.loads(open('gpurun_out/lmab_llama_$i.jsonl').read().strip().splitlines()[-1]); print(d['tokens_per_s'])")"
done
for v in PLX_ADAMW_WIDE=1 PLX_ADAMW_WIDE=0 PLX_ADAMW_WIDE=1 PLX_ADAMW_WIDE=0; do
  i=$((i + 1))
  env $v timeout -k 10 300 python scripts/bench_suite.py --only lm_gpt2 --quick > gpurun_out/lmab_gpt2_$i.jsonl 2> gpurun_out/lmab_gpt2_$i.err || { echo "variant '$v' failed"; tail -5 gpurun_out/lmab_gpt2_$i.err; exit 1; }
  echo "gpt2 [$v] $(python -c "import json; d=json.loads(open('gpurun_out/lmab_gpt2_$i.jsonl').read().strip().splitlines()[-1]); print(d['tokens_per_s'])")"
done
