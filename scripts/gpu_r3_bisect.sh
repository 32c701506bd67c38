#!/bin/bash
# round 3: bisect the ResNet bench regression over round-3 commits; PMC passes on the LM GEMM
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['train_images_per_s'])" "$1" "$2"; }
rc=0
for sha in db853c3 585c031 37df242; do
  (cd old_r2/bis_$sha && timeout -k 10 400 python bench.py --steps 3 --warmup 1 > ../../gpurun_out/bis_$sha.json 2> ../../gpurun_out/bis_$sha.err) || { rc=1; break; }
  summ gpurun_out/bis_$sha.json $sha || { rc=1; break; }
done
[ $rc = 0 ] \
&& timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d /tmp/gp1 -o run -- python scripts/gemm_one.py > gpurun_out/pmc/g1.log 2>&1 \
&& python scripts/pmc_summary.py $(ls /tmp/gp1/*/run_counter_collection.csv /tmp/gp1/run_counter_collection.csv 2>/dev/null | head -1) --match gemm256 > gpurun_out/pmc/g1.jsonl \
&& timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --output-format csv -d /tmp/gp2 -o run -- python scripts/gemm_one.py > gpurun_out/pmc/g2.log 2>&1 \
&& python scripts/pmc_summary.py $(ls /tmp/gp2/*/run_counter_collection.csv /tmp/gp2/run_counter_collection.csv 2>/dev/null | head -1) --match gemm256 > gpurun_out/pmc/g2.jsonl
rc=$?
echo "exit $rc"
exit $rc
