#!/bin/bash
# PMC passes over one LM GEMM shape: the kernel's schedules vs hipBLASLt (each counter set a KILL-limited run)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-gpmc}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  rm -rf /tmp/plx_pmc
  timeout -s KILL 90 rocprofv3 --pmc $set -d /tmp/plx_pmc -o run --output-format csv -- python3 scripts/gemm_micro.py 5 ${SHAPE:-4096 28672 4096} ${SCHEDS:-8,5,7} > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  f=$(find /tmp/plx_pmc -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" > gpurun_out/${TAG}_pmc$i.jsonl
  cut -c1-700 gpurun_out/${TAG}_pmc$i.jsonl
done
