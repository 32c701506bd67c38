#!/bin/bash
# Batch-generator rewrite: GPU tests, generator timing, then bench A/B of where the next batch is generated
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4synth_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4synth_pytest.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 120 python scripts/synth_time.py new > gpurun_out/r4synth_time.jsonl || exit 1
cat gpurun_out/r4synth_time.jsonl
AB_LIST="PLX_PREFETCH_AT=start;;PLX_PREFETCH_AT=start;PLX_PREFETCH_AT=end" TAG=r4pf bash scripts/gpu_ab_multi.sh
