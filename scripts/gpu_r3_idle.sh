#!/bin/bash
# round 3: where does the bench's time go (executor idle / in rounds / D2H sync), HEAD vs db853c3
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/idle_head.json 2> gpurun_out/idle_head.err \
&& python -c "import json; d=json.load(open('gpurun_out/idle_head.json')); print('head', d['value'], d['train_images_per_s'], d['per_rank'])" \
&& (cd old_r2/bis_db853c3 && timeout -k 10 400 python bench.py --steps 3 --warmup 1 > ../../gpurun_out/idle_r3a.json 2> ../../gpurun_out/idle_r3a.err) \
&& grep WSTATS gpurun_out/idle_r3a.err && python -c "import json; d=json.loads([l for l in open('gpurun_out/idle_r3a.json') if l.startswith('{')][-1]); print('db853c3', d['value'], d['train_images_per_s'])"
rc=$?
echo "exit $rc"
exit $rc
