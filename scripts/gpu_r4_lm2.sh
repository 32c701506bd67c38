#!/bin/bash
# Round 4: why the all-kernel LM step is slower than the isolated GEMM bench predicts -- the bench with operands
# streamed from HBM (--cold) and hot, and the hipBLASLt-mode kernel trace of the Llama step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/gemm_bench.py --models ${MODELS:-llama,gpt2} --waves 8,table,7,5 --cold 4 \
  > gpurun_out/r4g_cold.jsonl 2> gpurun_out/r4g_cold.err || { tail -20 gpurun_out/r4g_cold.err; exit 1; }
tail -1 gpurun_out/r4g_cold.jsonl
timeout -k 10 400 python scripts/gemm_bench.py --models ${MODELS:-llama,gpt2} --waves 8,table,7,5 \
  > gpurun_out/r4g_hot.jsonl 2> gpurun_out/r4g_hot.err || { tail -20 gpurun_out/r4g_hot.err; exit 1; }
tail -1 gpurun_out/r4g_hot.jsonl
PLX_LM_GEMM=0 TAG=r4lmprof_llama_hipblaslt WHICH=lm_llama8b bash scripts/gpu_lm_prof.sh > /dev/null || exit 1
head -14 gpurun_out/r4lmprof_llama_hipblaslt_kernels.md
