#!/bin/bash
# Round 4: conv kernel A/B on the ResNet-50 3x3 shapes (scripts/conv_ab.py), then optional PMC passes of one variant.
#   VARIANTS=base,tap_inner ROUNDS=7 PASSES=fwd,dgrad SHAPES=all PMC=0 scripts/gpu_r4_conv.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4conv}
timeout -k 10 300 python -u scripts/conv_ab.py "${VARIANTS:-base,tap_inner}" "${ROUNDS:-7}" "${PASSES:-fwd,dgrad}" \
  "${SHAPES:-all}" > gpurun_out/${TAG}_ab.jsonl 2> gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
cat gpurun_out/${TAG}_ab.jsonl
if [ "${PMC:-0}" != "0" ]; then
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i + 1))
    rm -rf /tmp/plx_pmc
    timeout -s KILL 120 rocprofv3 --pmc $set -d /tmp/plx_pmc -o run --output-format csv -- python3 scripts/conv_ab.py "${PMC_VARIANT:-base}" 1 "${PMC_PASS:-fwd}" "${PMC_SHAPES:-s1}" > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_pmc$i.log; continue; }
    f=$(find /tmp/plx_pmc -name '*counter_collection.csv' | head -1)
    python scripts/pmc_summary.py "$f" --match gemm_nt > gpurun_out/${TAG}_pmc$i.jsonl
    cut -c1-900 gpurun_out/${TAG}_pmc$i.jsonl
  done
fi
