#!/bin/bash
# round 3: ping-pong LM GEMM numerics + speed; ResNet bench A/B: HEAD vs the round-2 tree vs HEAD unpinned
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['train_images_per_s'], d.get('cpus_pinned'))" "$1" "$2"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_pytest.log 2>&1 \
&& echo "gemm tests ok" \
&& timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench3.jsonl 2> gpurun_out/gemm_bench3.err \
&& echo "gemm bench ok" \
&& timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/abr_head.json 2> gpurun_out/abr_head.err \
&& summ gpurun_out/abr_head.json head \
&& (cd old_r2 && timeout -k 10 400 python bench.py --steps 3 --warmup 1 > ../gpurun_out/abr_r2.json 2> ../gpurun_out/abr_r2.err) \
&& summ gpurun_out/abr_r2.json r2 \
&& PLX_BENCH_PIN=0 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/abr_nopin.json 2> gpurun_out/abr_nopin.err \
&& summ gpurun_out/abr_nopin.json nopin
rc=$?
echo "exit $rc"
tail -3 gpurun_out/gemm_pytest.log
exit $rc
