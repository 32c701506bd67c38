#!/bin/bash
# Weight-gradient kernels (scripts/wgrad_bench.py) under rocprofv3 PMC passes, each counter set a run of its own
# (KILL-limited); SHAPES = wgrad_bench shape indices, VARIANT = v1 / v2.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
TAG=${TAG:-wpmc}
SHAPES=${SHAPES:-9,17,18}
VARIANT=${VARIANT:-v2}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  rm -rf /tmp/plx_pmc
  timeout -s KILL 150 rocprofv3 --pmc $set -d /tmp/plx_pmc -o run --output-format csv -- python3 scripts/wgrad_bench.py --variants $VARIANT --shapes $SHAPES --rounds 1 --reps 3 --check 0 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  f=$(find /tmp/plx_pmc -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" --match _kernel > gpurun_out/${TAG}_pmc$i.jsonl
  cut -c1-700 gpurun_out/${TAG}_pmc$i.jsonl
done
