#!/bin/bash
# Same-box A/B of two builds of one native library (no rebuild on the box): targeted GPU tests with build A,
# then bench.py interleaved A B A B by swapping the .so in place.
# Usage: LIB=plx_bn TESTS="tests/test_gpu_bn.py" bash scripts/ab_lib.sh   (expects lib<LIB>_new.so / _old.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/ab
D=polyaxon_amd/_native
STEPS=${STEPS:-13}
WARM=${WARM:-2}
cp $D/lib${LIB}_new.so $D/lib${LIB}.so
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?
  tail -3 gpurun_out/ab/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for v in new old; do
    cp $D/lib${LIB}_${v}.so $D/lib${LIB}.so
    timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARM > gpurun_out/ab/b_${round}_${v}.json 2> gpurun_out/ab/b_${round}_${v}.err; rc=$?
    if [ $rc -ne 0 ]; then echo "bench [$v] failed rc=$rc"; tail -5 gpurun_out/ab/b_${round}_${v}.err; exit $rc; fi
    python - "$v" gpurun_out/ab/b_${round}_${v}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"[{sys.argv[1]}] {d['value']:.0f} trials/h  {d['ms_per_step']:.1f} ms/trial  {d['train_images_per_s']:.0f} img/s  best_loss {d['best_loss']}")
PY
  done
done
cp $D/lib${LIB}_new.so $D/lib${LIB}.so
