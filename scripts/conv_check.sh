set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/cbuild.log 2>&1 \
&& echo "== tests" && timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -x -q ${PYTEST_ARGS:-} > gpurun_out/ctest.log 2>&1; rc=$?
tail -30 gpurun_out/ctest.log
if [ $rc -eq 0 ]; then
  echo "== diag" && PYTHONPATH=. timeout -k 10 400 python scripts/diag_conv_gemm.py > gpurun_out/cdiag.log 2>&1; rc=$?
  cat gpurun_out/cdiag.log | grep -v amdgpu.ids
fi
exit $rc
