#!/bin/bash
# Llama-3 8B (or WHICH=lm_gpt2) tokens/s for several env variants back to back (AB_LIST ';'-separated)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-lmab}
WHICH=${WHICH:-lm_llama8b}
i=0
IFS=';' read -ra VARIANTS <<< "${AB_LIST:-}"
for v in "${VARIANTS[@]}"; do
  i=$((i + 1))
  env $v timeout -k 10 500 python scripts/bench_suite.py --only $WHICH --quick > gpurun_out/${TAG}_$i.jsonl 2> gpurun_out/${TAG}_$i.err || { echo "variant '$v' failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  echo "[$v] $(python -c "import json; d=json.loads(open('gpurun_out/${TAG}_$i.jsonl').read().strip().splitlines()[-1]); print(d.get('tokens_per_s'), d.get('loss'), d.get('error', '')[-200:])")"
done
