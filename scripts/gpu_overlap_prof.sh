#!/bin/bash
# Price the weight-gradient side stream: kernel traces of the bench step with the side stream (default) and with every
# weight gradient inline (PLX_WGRAD_STREAM=0) or the step replayed as a hipGraph (MODES="graph"), each split into
# forward / backward per stream (scripts/step_phases.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ovl}
for mode in ${MODES:-side inline}; do
  rm -rf /tmp/plx_prof_$mode
  if [ $mode = inline ]; then export PLX_WGRAD_STREAM=0; fi
  if [ $mode = graph ]; then export PLX_BENCH_GRAPH=1; fi
  timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/plx_prof_$mode -o run --output-format csv -- python bench.py --steps ${STEPS:-1} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_$mode.log 2>&1 || { echo "prof $mode failed"; tail -5 gpurun_out/${TAG}_$mode.log; exit 1; }
  trace=$(ls /tmp/plx_prof_$mode/*/run_kernel_trace.csv /tmp/plx_prof_$mode/run_kernel_trace.csv 2>/dev/null | head -1)
  python scripts/step_phases.py "$trace" --steps 20 > gpurun_out/${TAG}_${mode}_phases.md || exit 1
  python scripts/prof_summary.py "$trace" --steps 20 --top 45 --markdown > gpurun_out/${TAG}_${mode}_steady_state.md || exit 1
  echo "== $mode"; head -6 gpurun_out/${TAG}_${mode}_phases.md
done
