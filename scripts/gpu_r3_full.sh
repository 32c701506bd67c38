#!/bin/bash
# round 3: GPU test suite, Hyperband vs ASHA bench at the same target, rocprofv3 steady-state profile
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['train_images_per_s'], 'ttt', d['wall_clock_to_target_s'], 'best', d['sweep_best_loss'], d['loss_by_units'], d['per_rank'][0]['elapsed_s'])" "$1" "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_pytest.log 2>&1 \
&& tail -3 gpurun_out/r3_gpu_pytest.log \
&& timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r3_hb.json 2> gpurun_out/r3_hb.err \
&& summ gpurun_out/r3_hb.json hb \
&& timeout -k 10 400 python bench.py --steps 3 --warmup 1 --search asha > gpurun_out/r3_asha.json 2> gpurun_out/r3_asha.err \
&& summ gpurun_out/r3_asha.json asha \
&& PROF_TAG=r3_resnet50_hb STEPS=2 bash scripts/prof_only.sh
rc=$?
echo "exit $rc"
tail -5 gpurun_out/r3_gpu_pytest.log
exit $rc
