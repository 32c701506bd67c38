#!/bin/bash
# A/B of NT GEMM variants on the ResNet-50 layer shapes (scripts/roofline_resnet.py) + profile of a bench run
# summarised on the box (the raw trace is too large to bring back).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=${ONLY:-conv}
timeout -k 10 300 python -c "from polyaxon_amd.ops import _native; _native.build_all()" > gpurun_out/abbuild.log 2>&1 \
&& timeout -k 10 300 python scripts/roofline_resnet.py --only "$ONLY" --nt-single-stage 0 > gpurun_out/ab_nt_base.jsonl 2> gpurun_out/ab_nt_base.err \
&& timeout -k 10 300 python scripts/roofline_resnet.py --only "$ONLY" --nt-single-stage 1 > gpurun_out/ab_nt_new.jsonl 2> gpurun_out/ab_nt_new.err \
&& timeout -k 10 300 python scripts/roofline_resnet.py --only "$ONLY" --nt-single-stage 0 > gpurun_out/ab_nt_base2.jsonl 2>> gpurun_out/ab_nt_base.err \
&& if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof.log 2>&1 \
  && python scripts/prof_summary.py "$(find /tmp/prof -name "*kernel_trace.csv" | head -1)" --steps 40 --markdown > gpurun_out/prof_summary.md 2>&1
fi
rc=$?
echo "exit $rc"
exit $rc
