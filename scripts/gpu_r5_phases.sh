#!/bin/bash
# Kernel traces of the ResNet-50 bench per weight-gradient variant, summarised on the box: step phases (forward /
# backward, per-stream busy and union) and the steady-state kernel table.  CONFIGS: space-separated NAME=ENV pairs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
for cfg in ${CONFIGS:-v1:PLX_TN_V2=0 v2s:PLX_TN_V2=1,64 v2s_inline:PLX_TN_V2=1,64,PLX_WGRAD_STREAM=0}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  rm -rf /tmp/plx_prof
  echo "== $name ($envs)"
  env ${envs//,PLX/ PLX} timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/plx_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/ph_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ph_$name.log; exit 1; }
  trace=$(ls /tmp/plx_prof/*/run_kernel_trace.csv /tmp/plx_prof/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/step_phases.py "$trace" --steps 20 --markdown > gpurun_out/ph_${name}_phases.md
  python3 scripts/prof_summary.py "$trace" --steps 20 --top 30 --markdown > gpurun_out/ph_${name}_steady.md
  head -30 gpurun_out/ph_${name}_phases.md
done
