#!/bin/bash
# Same-box A/B: build, targeted GPU tests, optional diag, then bench variants interleaved (A B A B).
# Usage: VARIANTS="|--miopen-1x1" TESTS="tests/test_gpu_conv.py" bash scripts/ab_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/ab
STEPS=${STEPS:-2}
WARM=${WARM:-1}
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/ab/build.log 2>&1 || { echo build failed; tail gpurun_out/ab/build.log; exit 1; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -m pytest $TESTS -x -q > gpurun_out/ab/tests.log 2>&1; rc=$?
  tail -5 gpurun_out/ab/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${DIAG:-}" ]; then
  timeout -k 10 400 python $DIAG > gpurun_out/ab/diag.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/ab/diag.log | tail -25
  [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra VS <<< "${VARIANTS:-}"
for round in 1 2; do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    # a variant is bench flags and/or leading NAME=VALUE environment settings (A/B knobs)
    timeout -k 10 600 env $v python bench.py --steps $STEPS --warmup $WARM > gpurun_out/ab/b_${round}_${i}.json 2> gpurun_out/ab/b_${round}_${i}.err; rc=$?
    if [ $rc -ne 0 ]; then echo "bench [$v] failed rc=$rc"; tail -5 gpurun_out/ab/b_${round}_${i}.err; exit $rc; fi
    python - "$v" gpurun_out/ab/b_${round}_${i}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"[{sys.argv[1] or 'default'}] {d['value']:.0f} trials/h  {d['train_images_per_s']:.0f} img/s  best_loss {d['best_loss']}")
PY
  done
done
