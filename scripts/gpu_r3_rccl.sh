#!/bin/bash
# round 3: does a live RCCL communicator slow the launch path? + bench with the communicator created late
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/launch_overhead.py > gpurun_out/launch_overhead.json 2> gpurun_out/launch_overhead.err \
&& cat gpurun_out/launch_overhead.json \
&& timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/rccl_late.json 2> gpurun_out/rccl_late.err \
&& python -c "import json; d=json.load(open('gpurun_out/rccl_late.json')); print('late', d['value'], d['train_images_per_s'], d['per_rank'])" \
&& PLX_BENCH_RCCL=0 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/rccl_off.json 2> gpurun_out/rccl_off.err \
&& python -c "import json; d=json.load(open('gpurun_out/rccl_off.json')); print('off', d['value'], d['train_images_per_s'])"
rc=$?
echo "exit $rc"
exit $rc
