#!/bin/bash
# Round 4: LM tokens/s at the final dispatch (GPT-2 padded vs unpadded vocabulary, Llama-3 8B), then the RCCL
# communicator A/B with base / early kernel traces
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r4final_lm bash scripts/gpu_lm_tokens.sh || exit 1
PLX_VOCAB_MULTIPLE=1 timeout -k 10 300 python scripts/bench_suite.py --only lm_gpt2 --quick > gpurun_out/r4final_lm_gpt2_unpadded.jsonl \
  2> gpurun_out/r4final_lm_gpt2_unpadded.err || exit 1
tail -1 gpurun_out/r4final_lm_gpt2_unpadded.jsonl | cut -c1-300
bash scripts/gpu_r4_rccl.sh || exit 1
