#!/bin/bash
# Interleaved A/B of env-var knobs on the ResNet-50 layer shapes: VARIANTS="A=1 A=2 A=1 A=2" runs
# scripts/roofline_resnet.py --only "$ONLY" once per variant (own process, same device), output ab_<variant>_r<i>.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=${ONLY:-bn}
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/abbuild.log 2>&1 || exit 1
i=0
for v in $VARIANTS; do
  i=$((i+1))
  env "$v" timeout -k 10 300 python scripts/roofline_resnet.py --only "$ONLY" > "gpurun_out/ab_${v}_r$i.jsonl" 2> "gpurun_out/ab_${v}_r$i.err" || { echo "$v failed"; exit 1; }
  echo "$v round $i done"
done
echo "exit 0"
