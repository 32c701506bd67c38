#!/bin/bash
# attention microbenchmark (HIP flash attention at the LM shapes), optional PLX_ATTN_* knobs from the caller
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-attn}
timeout -k 10 300 python -u scripts/bench_attention.py hip ${SHAPES:-} > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.err
rc=$?
cat gpurun_out/${TAG}.jsonl
tail -5 gpurun_out/${TAG}.err
exit $rc
