#!/bin/bash
# Kernel totals of the LM training step (bench_suite lm_llama8b / lm_gpt2, --quick) under rocprofv3 --kernel-trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-lmprof}
WHICH=${WHICH:-lm_llama8b}
rm -rf /tmp/plx_lmprof
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/plx_lmprof -o run -- python3 scripts/bench_suite.py --only $WHICH --quick > gpurun_out/${TAG}.log 2>&1 || { tail -5 gpurun_out/${TAG}.log; exit 1; }
db=$(find /tmp/plx_lmprof -name '*.db' | head -1)
python scripts/kernel_totals.py "$db" --top 40 > gpurun_out/${TAG}_kernels.md
python scripts/lm_step_streams.py "$db" --steps 2 > gpurun_out/${TAG}_streams.md || true
cat gpurun_out/${TAG}_streams.md
if [ -n "${NEIGHBORS:-}" ]; then  # comma-separated kernel-name patterns: who launches them
  IFS=',' read -ra pats <<< "$NEIGHBORS"
  for p in "${pats[@]}"; do python scripts/kernel_neighbors.py "$db" "$p" --n 2 ${NEIGHBORS_ARGS:---skip 40}; done > gpurun_out/${TAG}_neighbors.txt
  cat gpurun_out/${TAG}_neighbors.txt
fi
grep tokens_per_s gpurun_out/${TAG}.log | tail -1 | cut -c1-200
head -25 gpurun_out/${TAG}_kernels.md
