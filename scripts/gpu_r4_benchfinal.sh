#!/bin/bash
# Round 4 final tree: the driver-shaped bench (20 sweeps after 5 warm-up), then a kernel-trace profile of 2 sweeps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r4final_bench.json 2> gpurun_out/r4final_bench.err || { tail -20 gpurun_out/r4final_bench.err; exit 1; }
tail -1 gpurun_out/r4final_bench.json | cut -c1-400
PROF_TAG=r4final_resnet50_hb STEPS=2 bash scripts/prof_only.sh || exit 1
head -14 gpurun_out/r4final_resnet50_hb_steady_state.md
