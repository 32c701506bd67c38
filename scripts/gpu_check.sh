#!/bin/bash
# GPU-box check: build, smoke, gpu tests, bench, rocprof kernel trace. Each GPU step has its own timeout
# and the chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-13}
WARM=${WARM:-2}
echo "== build" && timeout -k 10 300 python __graft_entry__.py > gpurun_out/build.log 2>&1 \
&& echo "== smoke" && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 900 python bench.py --steps $STEPS --warmup $WARM ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& cat gpurun_out/bench.json \
&& echo "== rocprof" && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 \
&& echo "== gpt2" && timeout -k 10 600 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 20 --log_every 100 > gpurun_out/gpt2.json 2> gpurun_out/gpt2.err \
&& cat gpurun_out/gpt2.json \
&& echo "== done"
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_gpu.log
exit $rc
