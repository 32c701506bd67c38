#!/bin/bash
# Round 4: grouped tile order for the LM GEMM kernels (L2 reuse) -- numerics, then groups 1 / 4 / 8 vs hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r4grp_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4grp_tests.log; exit 1; }
tail -1 gpurun_out/r4grp_tests.log
timeout -k 10 500 python scripts/gemm_bench.py --waves 8,5 --groups 1,4,8 > gpurun_out/r4grp_bench.jsonl 2> gpurun_out/r4grp_bench.err \
  || { tail -20 gpurun_out/r4grp_bench.err; exit 1; }
tail -1 gpurun_out/r4grp_bench.jsonl
SHAPE="4096 28672 4096" SCHEDS=8,5 TAG=r4grp bash scripts/gpu_gemm_pmc.sh > /dev/null || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r4grp_pmc2.jsonl"):
    d = json.loads(l)
    if "TCC_HIT_sum" in d and d.get("SQ_INSTS_MFMA"):
        h, m = d["TCC_HIT_sum"], d["TCC_MISS_sum"]
        print(d["kernel"][:60], "L2 hit", round(h / (h + m), 3))
PY
