#!/bin/bash
# Round 4: LM path with every linear on gemm256 (per-shape schedules, padded GPT-2 vocabulary): GPU tests, tokens/s
# (default and the hipBLASLt A/B), kernel-trace profiles of both models
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_models.py tests/test_gpu_lm.py \
  > gpurun_out/r4lm_tests.log 2>&1 || { tail -40 gpurun_out/r4lm_tests.log; exit 1; }
tail -2 gpurun_out/r4lm_tests.log
TAG=r4lm bash scripts/gpu_lm_tokens.sh || exit 1
PLX_LM_GEMM=0 TAG=r4lm_hipblaslt bash scripts/gpu_lm_tokens.sh || exit 1
TAG=r4lm_again bash scripts/gpu_lm_tokens.sh || exit 1
TAG=r4lmprof_gpt2 WHICH=lm_gpt2 bash scripts/gpu_lm_prof.sh > /dev/null || exit 1
TAG=r4lmprof_llama WHICH=lm_llama8b bash scripts/gpu_lm_prof.sh > /dev/null || exit 1
grep -c Cijk gpurun_out/r4lmprof_gpt2_kernels.md gpurun_out/r4lmprof_llama_kernels.md || true
head -12 gpurun_out/r4lmprof_gpt2_kernels.md; head -12 gpurun_out/r4lmprof_llama_kernels.md
