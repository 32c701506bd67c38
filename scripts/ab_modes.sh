#!/bin/bash
# Interleaved A/B of the NT GEMM single-buffer modes (plx_set_nt_single_stage) on the ResNet-50 layer shapes:
# MODES rounds in one box session, each a separate scripts/roofline_resnet.py process (same device).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=${ONLY:-conv}
MODES=${MODES:-"1 2 3 1 2 3"}
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/abbuild.log 2>&1 || exit 1
i=0
for m in $MODES; do
  i=$((i+1))
  timeout -k 10 300 python scripts/roofline_resnet.py --only "$ONLY" --nt-single-stage $m > gpurun_out/ab_mode${m}_r$i.jsonl 2> gpurun_out/ab_mode${m}_r$i.err || { echo "mode $m failed"; exit 1; }
  echo "mode $m round $i done"
done
echo "exit 0"
