#!/bin/bash
# Round 4: config-4 (gpt2_bo) bench, config-5 DP=1 through polyflow, then the RCCL-communicator A/B (each step under
# its own time limit; stops at the first failure)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${BO:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py --config gpt2_bo --steps ${BO_STEPS:-1} --warmup 1 > gpurun_out/r4_gpt2_bo.json 2> gpurun_out/r4_gpt2_bo.err || { tail -30 gpurun_out/r4_gpt2_bo.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_gpt2_bo.json').read().strip().splitlines()[-1]); print('gpt2_bo', {k: d[k] for k in ('value','trials','best_loss','ms_per_step','train_images_per_s','per_rank')})"
fi
if [ "${BOP:-1}" = "1" ]; then  # the same BO group in process mode (a fresh trainer process per trial)
  timeout -k 10 1000 python scripts/gpt2_bo_process.py > gpurun_out/r4_gpt2_bo_process.json 2> gpurun_out/r4_gpt2_bo_process.err \
    || { tail -30 gpurun_out/r4_gpt2_bo_process.err; exit 1; }
  cat gpurun_out/r4_gpt2_bo_process.json
fi
if [ "${C5:-1}" = "1" ]; then
  bash scripts/gpu_r4_config5.sh || exit 1
fi
if [ "${RCCL:-1}" = "1" ]; then
  bash scripts/gpu_r4_rccl.sh || exit 1
fi
