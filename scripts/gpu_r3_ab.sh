#!/bin/bash
# round 3: bench A/B (CPU pinning, RCCL communicator) + PMC passes on the 3x3 convolution kernels
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
STEPS=${STEPS:-3}
run_bench() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps $STEPS --warmup 1 --target 0.02 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || return 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', d['value'], d['train_images_per_s'], d['cpus_pinned'], d['wall_clock_to_target_s'], d['sweep_best_loss'])"
}
run_bench default PLX_X=1 \
&& run_bench pinforce PLX_BENCH_PIN=force \
&& run_bench norccl PLX_BENCH_RCCL=0 \
&& run_bench default2 PLX_X=1 \
&& echo "== pmc pass 1" \
&& timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d /tmp/pmc1 -o run -- python scripts/roofline_resnet.py --only s3.j.conv2,s2.j.conv2 --reps 2 > gpurun_out/pmc/p1.log 2>&1 \
&& python scripts/pmc_summary.py $(ls /tmp/pmc1/*/run_counter_collection.csv /tmp/pmc1/run_counter_collection.csv 2>/dev/null | head -1) --match gemm > gpurun_out/pmc/p1.jsonl \
&& echo "== pmc pass 2" \
&& timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --output-format csv -d /tmp/pmc2 -o run -- python scripts/roofline_resnet.py --only s3.j.conv2,s2.j.conv2 --reps 2 > gpurun_out/pmc/p2.log 2>&1 \
&& python scripts/pmc_summary.py $(ls /tmp/pmc2/*/run_counter_collection.csv /tmp/pmc2/run_counter_collection.csv 2>/dev/null | head -1) --match gemm > gpurun_out/pmc/p2.jsonl
rc=$?
echo "exit $rc"
exit $rc
