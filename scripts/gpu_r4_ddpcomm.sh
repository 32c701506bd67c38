#!/bin/bash
# Bucket all-reduces on the framework RCCL communicator vs ProcessGroupNCCL: GPU test, then GPT-2 world-1 A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4ddpc_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4ddpc_pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in ":--world1_collectives all" "PLX_DDP_COMM=rccl:--world1_collectives all" ":" "PLX_DDP_COMM=rccl:--world1_collectives all"; do
  i=$((i + 1))
  envs=${v%%:*}; args=${v#*:}
  env $envs timeout -k 10 300 python -m polyaxon_amd.trainers lm --model gpt2_125m --bs 16 --seq 1024 --steps 40 $args > gpurun_out/r4ddpc_$i.json 2> gpurun_out/r4ddpc_$i.err || { tail -20 gpurun_out/r4ddpc_$i.err; exit 1; }
  echo "[$envs $args] $(python -c "import json; d=json.loads(open('gpurun_out/r4ddpc_$i.json').read().strip().splitlines()[-1]); print(d['tokens_per_s'], d['loss'], d['bucket_launches'])")"
done
