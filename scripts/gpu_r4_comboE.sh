#!/bin/bash
# Round 4: LM tokens/s at the final dispatch (GPT-2 padded vs unpadded vocabulary, Llama-3 8B), then the Llama step
# bare vs a world-1 nccl PG + metric communicator vs + every bucket all-reduce
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r4final_lm bash scripts/gpu_lm_tokens.sh || exit 1
PLX_VOCAB_MULTIPLE=1 timeout -k 10 300 python scripts/bench_suite.py --only lm_gpt2 --quick > gpurun_out/r4final_lm_gpt2_unpadded.jsonl \
  2> gpurun_out/r4final_lm_gpt2_unpadded.err || exit 1
tail -1 gpurun_out/r4final_lm_gpt2_unpadded.jsonl | cut -c1-300
T="python -m polyaxon_amd.trainers lm --model llama3_8b --bs 1 --seq 4096 --steps 20 --lr 3e-4 --log_every 5"
for v in "" "--world1_collectives metric" "--world1_collectives all" ""; do
  timeout -k 10 400 $T $v > gpurun_out/r4e_c5.log 2>&1 || { tail -20 gpurun_out/r4e_c5.log; exit 1; }
  echo "llama [$v] $(grep '^{' gpurun_out/r4e_c5.log | tail -1 | cut -c1-200)"
done
