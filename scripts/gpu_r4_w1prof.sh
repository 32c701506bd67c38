#!/bin/bash
# GPT-2 trainer with and without world-1 bucket all-reduces under rocprofv3 kernel traces (where do 12 ms/step go?)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in base all; do
  args=""; [ $tag = all ] && args="--world1_collectives all"
  rm -rf /tmp/plx_w1_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/plx_w1_$tag -o run --output-format csv -- python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 20 $args > gpurun_out/r4w1_$tag.log 2>&1 || { tail -20 gpurun_out/r4w1_$tag.log; exit 1; }
  stats=$(ls /tmp/plx_w1_$tag/*/run_kernel_stats.csv /tmp/plx_w1_$tag/run_kernel_stats.csv 2>/dev/null | head -1)
  trace=$(ls /tmp/plx_w1_$tag/*/run_kernel_trace.csv /tmp/plx_w1_$tag/run_kernel_trace.csv 2>/dev/null | head -1)
  cp "$stats" gpurun_out/r4w1_${tag}_kernel_stats.csv
  python scripts/prof_summary.py "$trace" --steps 10 --top 25 --markdown > gpurun_out/r4w1_${tag}_steady_state.md
  tail -1 gpurun_out/r4w1_$tag.log | cut -c1-200
done
python scripts/kernel_stats_diff.py gpurun_out/r4w1_base_kernel_stats.csv gpurun_out/r4w1_all_kernel_stats.csv --top 15
head -12 gpurun_out/r4w1_all_steady_state.md
