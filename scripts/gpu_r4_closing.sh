#!/bin/bash
# End of round 4: GPU suite + smoke, the LM trainer's planned buckets on the RCCL path (world-1 collectives), then the
# driver-shaped bench (20 sweeps after 5 warm-up) and a kernel-trace profile of 2 sweeps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4close_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4close_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4close_smoke.log 2>&1 || { tail -20 gpurun_out/r4close_smoke.log; exit 1; }
tail -1 gpurun_out/r4close_smoke.log
timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 20 --world1_collectives all > gpurun_out/r4close_gpt2_auto_buckets.json 2> gpurun_out/r4close_gpt2_auto_buckets.err || { tail -20 gpurun_out/r4close_gpt2_auto_buckets.err; exit 1; }
tail -1 gpurun_out/r4close_gpt2_auto_buckets.json | cut -c1-500
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r4close_bench.json 2> gpurun_out/r4close_bench.err || { tail -20 gpurun_out/r4close_bench.err; exit 1; }
tail -1 gpurun_out/r4close_bench.json | cut -c1-400
PROF_TAG=r4close_resnet50_hb STEPS=2 bash scripts/prof_only.sh || exit 1
head -14 gpurun_out/r4close_resnet50_hb_steady_state.md
