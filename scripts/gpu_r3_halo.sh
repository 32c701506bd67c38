#!/bin/bash
# round 3: build, gpu tests (incl. the halo conv tests), 3x3 roofline with halo on/off, benches
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-3}
echo "== pytest gpu conv" && timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1 \
&& tail -1 gpurun_out/pytest_conv.log \
&& echo "== roofline 3x3 halo" && PLX_HALO=1 timeout -k 10 300 python scripts/roofline_resnet.py --only conv2 --md gpurun_out/roof_halo1.md > gpurun_out/roof_halo1.jsonl 2>&1 \
&& echo "== roofline 3x3 gather" && PLX_HALO=0 timeout -k 10 300 python scripts/roofline_resnet.py --only conv2 --md gpurun_out/roof_halo0.md > gpurun_out/roof_halo0.jsonl 2>&1 \
&& echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& tail -1 gpurun_out/pytest_gpu.log \
&& echo "== bench hyperband" && timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench_hb.json 2> gpurun_out/bench_hb.err \
&& cat gpurun_out/bench_hb.json \
&& echo "== bench hyperband halo off" && PLX_HALO=0 timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench_hb0.json 2> gpurun_out/bench_hb0.err \
&& cat gpurun_out/bench_hb0.json \
&& echo "== bench asha" && timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 --search asha > gpurun_out/bench_asha.json 2> gpurun_out/bench_asha.err \
&& cat gpurun_out/bench_asha.json
rc=$?
echo "exit $rc"
exit $rc
