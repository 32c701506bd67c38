set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/diag_bo1000.py 1000 > gpurun_out/diag_bo1000.log 2>&1 \
&& timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gp.log 2>&1 \
&& timeout -k 10 600 python scripts/bench_suite.py --only bo --bo-backends hip > gpurun_out/suite_bo.jsonl 2> gpurun_out/suite_bo.err
rc=$?
cat gpurun_out/diag_bo1000.log | tail -20; tail -3 gpurun_out/pytest_gp.log; cat gpurun_out/suite_bo.jsonl
echo "exit $rc"; exit $rc
