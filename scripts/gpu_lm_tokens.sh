#!/bin/bash
# LM training tokens/s (GPT-2 125M, Llama-3 8B on one GPU) at the default dispatch (each run under its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-lm}
timeout -k 10 300 python scripts/bench_suite.py --only lm_gpt2 --quick > gpurun_out/${TAG}_gpt2.jsonl 2> gpurun_out/${TAG}_gpt2.err || exit 1
tail -1 gpurun_out/${TAG}_gpt2.jsonl | cut -c1-300
timeout -k 10 500 python scripts/bench_suite.py --only lm_llama8b --quick > gpurun_out/${TAG}_llama.jsonl 2> gpurun_out/${TAG}_llama.err || exit 1
tail -1 gpurun_out/${TAG}_llama.jsonl | cut -c1-300
