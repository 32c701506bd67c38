#!/bin/bash
# round 3: LM training tokens/s with the LM GEMM dispatch modes (auto = per-shape fastest, 1 = MFMA kernel, 0 = hipBLASLt)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rc=0
for m in auto 1 0; do
  PLX_LM_GEMM=$m timeout -k 10 300 python scripts/bench_suite.py --only lm_gpt2 --quick > gpurun_out/lm_gpt2_$m.jsonl 2> gpurun_out/lm_gpt2_$m.err || { rc=1; break; }
  echo "gpt2 $m $(python -c "import json; d=json.loads(open('gpurun_out/lm_gpt2_$m.jsonl').read().strip().splitlines()[-1]); print(d.get('tokens_per_s'), d.get('lm_gemm', {}).get('native_shapes'), d.get('lm_gemm', {}).get('shapes'), d.get('error', '')[-300:])")"
done
if [ $rc = 0 ]; then
for m in auto 0; do
  PLX_LM_GEMM=$m timeout -k 10 500 python scripts/bench_suite.py --only lm_llama8b --quick > gpurun_out/lm_llama_$m.jsonl 2> gpurun_out/lm_llama_$m.err || { rc=1; break; }
  echo "llama $m $(python -c "import json; d=json.loads(open('gpurun_out/lm_llama_$m.jsonl').read().strip().splitlines()[-1]); print(d.get('tokens_per_s'), d.get('ms_per_step'), d.get('lm_gemm', {}).get('native_shapes'), d.get('lm_gemm', {}).get('shapes'), d.get('error', '')[-300:])")"
done
fi
echo "exit $rc"
exit $rc
