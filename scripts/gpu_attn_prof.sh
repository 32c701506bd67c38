#!/bin/bash
# per-kernel times of the attention microbenchmark (rocprofv3 kernel trace, stats only)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-attn_prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o run -- python3 scripts/bench_attention.py hip ${SHAPES:-llama3_8b} > gpurun_out/${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}.log
f=$(find gpurun_out/${TAG} -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -15
exit $rc
