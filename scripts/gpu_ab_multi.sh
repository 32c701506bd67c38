#!/bin/bash
# Several bench variants back to back on one box (each its own process and time limit): AB_LIST is a ';'-separated
# list of env assignments ("" = default), e.g. AB_LIST='X=1;X=1 Y=2;'
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
i=0
IFS=';' read -ra VARIANTS <<< "${AB_LIST:-}"
for v in "${VARIANTS[@]}"; do
  i=$((i + 1))
  env $v timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "variant '$v' failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  echo "[$v] $(python -c "import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); print(d['value'], d.get('train_images_per_s'))")"
done
