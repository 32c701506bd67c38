#!/bin/bash
# Round 4: >= 10 sweeps each of the Hyperband and ASHA benches on one box (time-to-target distribution, ASHA sync)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in ${SEARCHES:-hyperband asha}; do
  timeout -k 10 600 python bench.py --search $s --steps ${SWEEPS:-10} --warmup 1 > gpurun_out/r4sw_$s.json 2> gpurun_out/r4sw_$s.err \
    || { tail -30 gpurun_out/r4sw_$s.err; exit 1; }
  tail -1 gpurun_out/r4sw_$s.json | cut -c1-600
done
