#!/bin/bash
# 3x3 conv microbenchmark timings, then rocprofv3 PMC passes (each counter set a run of its own, KILL-limited)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-cpmc}
timeout -k 10 120 python scripts/conv3x3_micro.py both 20 > gpurun_out/${TAG}_times.jsonl 2> gpurun_out/${TAG}_times.err || { tail -5 gpurun_out/${TAG}_times.err; exit 1; }
cat gpurun_out/${TAG}_times.jsonl
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  rm -rf /tmp/plx_pmc
  timeout -s KILL 120 rocprofv3 --pmc $set -d /tmp/plx_pmc -o run --output-format csv -- python3 scripts/conv3x3_micro.py ${PASS:-fwd} 5 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  f=$(find /tmp/plx_pmc -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" --match gemm_nt > gpurun_out/${TAG}_pmc$i.jsonl
  cut -c1-600 gpurun_out/${TAG}_pmc$i.jsonl
done
