#!/bin/bash
# One driver for every GPU-box job of this repository (run it through gpurun from the repo root):
#
#   bash scripts/gpu.sh MODE [args]
#
# MODE
#   tests [pytest targets]   pytest -m gpu (default: the whole suite), one process, per-test thread timeout
#   final                    the driver's round-end tiers on the in-tree .so files: pytest -m gpu, smoke(), bench.py
#   bench                    one bench.py run (BENCH_ARGS, default --steps 3 --warmup 1)
#   ab                       bench.py once per variant of AB_LIST (';'-separated env assignments, "" = defaults, in
#                            the order given: list A;B;A;B to interleave), one JSON line each in $TAG.jsonl; CMD
#                            replaces "bench.py $BENCH_ARGS" (any python argv printing a JSON line last, e.g.
#                            CMD="-m polyaxon_amd.trainers lm --model gpt2_125m"), and a variant may append arguments
#                            after a '|' ("PLX_X=1|--zero1")
#   ablib                    the same, swapping two builds of one library in place: LIB=plx_bn expects
#                            polyaxon_amd/_native/lib<LIB>_{new,old}.so, runs TESTS with "new", then new/old x ROUNDS
#                            (CMD as for ab)
#   prof                     rocprofv3 kernel trace of bench.py (BENCH_ARGS), summarised on the box: steady-state
#                            kernel table (prof_summary.py) and step phases (step_phases.py); AB_LIST as for ab;
#                            WINDOW=<kernel substring>: the launch sequence around it (trace_window.py); the
#                            all-stream idle intervals by neighbouring kernels (gap_report.py)
#   pmc CMD...               PMC passes over CMD (each counter set its own KILL-limited run, COUNTER_SETS ';'-separated,
#                            default: issue / LDS / MFMA / L2 sets), summarised by pmc_summary.py (MATCH = kernel filter)
#   py SCRIPT [args]         a python script under a time limit (LIMIT seconds), stdout to $TAG.out
#   suite                    the non-headline BASELINE configs (scripts/bench_suite.py, SUITE) + the GP kernel tests
#
# Every GPU step runs under its own `timeout -k 10`; the first failure ends the job (no retries).  Outputs land in
# gpurun_out/ (TAG prefixes the file names).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
MODE=${1:-tests}
[ $# -gt 0 ] && shift
TAG=${TAG:-$MODE}
O=gpurun_out/$TAG

fail() { echo "$1 failed (rc $2)"; [ -n "${3:-}" ] && tail -8 "$3"; exit "$2"; }

bench_line() {  # JSON line of a bench.py output file, with the variant label
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
keep = ("value", "ms_per_step", "train_images_per_s", "tokens_per_s", "best_loss", "control_device_footprint", "zero1",
        "world1_collectives", "bucket_launches", "buckets")
print(json.dumps({"variant": sys.argv[1], **{k: d[k] for k in keep if k in d}}))
PY
}

variants() {  # AB_LIST split on ';' into the array V
  IFS=';' read -ra V <<< "${AB_LIST:-}"
  [ ${#V[@]} -eq 0 ] && V=("")
}

case $MODE in
tests)
  if [ $# -gt 0 ]; then args=("$@"); else args=(tests -m gpu); fi
  timeout -k 10 ${LIMIT:-1000} python -u -m pytest "${args[@]}" -x -q --timeout 120 --timeout-method thread \
    > $O.log 2>&1 || fail pytest $? $O.log
  tail -2 $O.log ;;
final)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > ${O}_pytest.log 2>&1 \
    || fail pytest $? ${O}_pytest.log
  tail -2 ${O}_pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1 \
    || fail smoke $? ${O}_smoke.log
  tail -1 ${O}_smoke.log
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > ${O}_bench.json 2> ${O}_bench.err || fail bench $? ${O}_bench.err
  cut -c1-800 ${O}_bench.json ;;
bench)
  timeout -k 10 ${LIMIT:-900} python -u bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > $O.json 2> $O.err \
    || fail bench $? $O.err
  cut -c1-1500 $O.json ;;
ab)
  variants; : > $O.jsonl; i=0
  for v in "${V[@]}"; do
    i=$((i + 1)); e=${v%%|*}; extra=""; [ "$e" != "$v" ] && extra=${v#*|}
    env $e timeout -k 10 ${LIMIT:-600} python -u ${CMD:-bench.py ${BENCH_ARGS:---steps 3 --warmup 1}} $extra \
      > ${O}_$i.json 2> ${O}_$i.err || fail "variant '$v'" $? ${O}_$i.err
    bench_line "$v" ${O}_$i.json >> $O.jsonl
    tail -1 $O.jsonl
  done ;;
ablib)
  D=polyaxon_amd/_native
  cp $D/lib${LIB}_new.so $D/lib${LIB}.so
  if [ -n "${TESTS:-}" ]; then
    timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 \
      || fail tests $? ${O}_tests.log
    tail -2 ${O}_tests.log
  fi
  : > $O.jsonl
  for r in $(seq ${ROUNDS:-2}); do
    for v in new old; do
      cp $D/lib${LIB}_$v.so $D/lib${LIB}.so
      timeout -k 10 600 python -u ${CMD:-bench.py ${BENCH_ARGS:---steps 13 --warmup 2}} > ${O}_${r}_$v.json 2> ${O}_${r}_$v.err \
        || fail "bench [$v]" $? ${O}_${r}_$v.err
      bench_line "$v" ${O}_${r}_$v.json >> $O.jsonl
      tail -1 $O.jsonl
    done
  done
  cp $D/lib${LIB}_new.so $D/lib${LIB}.so ;;
prof)
  variants; i=0
  for v in "${V[@]}"; do
    i=$((i + 1)); rm -rf /tmp/plx_prof
    env $v timeout -k 10 ${LIMIT:-900} rocprofv3 --kernel-trace --stats -d /tmp/plx_prof -o run --output-format csv \
      -- python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1} > ${O}_$i.log 2>&1 || fail "prof '$v'" $? ${O}_$i.log
    trace=$(ls /tmp/plx_prof/*/run_kernel_trace.csv /tmp/plx_prof/run_kernel_trace.csv 2>/dev/null | head -1)
    stats=$(ls /tmp/plx_prof/*/run_kernel_stats.csv /tmp/plx_prof/run_kernel_stats.csv 2>/dev/null | head -1)
    [ -n "$stats" ] && cp "$stats" ${O}_${i}_kernel_stats.csv
    python3 scripts/prof_summary.py "$trace" --steps ${PROF_STEPS:-40} --top 40 --markdown > ${O}_${i}_steady_state.md
    python3 scripts/step_phases.py "$trace" --steps ${PROF_STEPS:-40} --markdown > ${O}_${i}_phases.md
    python3 scripts/gap_report.py "$trace" > ${O}_${i}_gaps.jsonl
    if [ -n "${WINDOW:-}" ]; then  # kernel sequence around a kernel (scripts/trace_window.py --match $WINDOW)
      python3 scripts/trace_window.py "$trace" --match "$WINDOW" --before ${WBEFORE:-20} --after ${WAFTER:-30} \
        > ${O}_${i}_window.txt
    fi
    echo "== [$v]"; head -25 ${O}_${i}_phases.md
  done ;;
apitrace)  # HIP API + kernel trace of bench.py: which API calls block the host, and the host's lead (api_blockers.py)
  rm -rf /tmp/plx_api
  timeout -k 10 ${LIMIT:-600} rocprofv3 --hip-trace --kernel-trace -d /tmp/plx_api -o run --output-format csv \
    -- python3 bench.py ${BENCH_ARGS:---steps 1 --warmup 0} > ${O}.log 2>&1 || fail "apitrace" $? ${O}.log
  api=$(find /tmp/plx_api -name 'run_hip_api_trace.csv' | head -1)
  trace=$(find /tmp/plx_api -name 'run_kernel_trace.csv' | head -1)
  timeout -k 10 300 python3 scripts/api_blockers.py "$api" "$trace" > ${O}_blockers.jsonl || fail blockers $? ${O}.log
  if [ -n "${WINDOW:-}" ]; then
    python3 scripts/trace_window.py "$trace" --api "$api" --match "$WINDOW" --occurrence ${WOCC:--2} \
      --before ${WBEFORE:-20} --after ${WAFTER:-40} > ${O}_window.txt
  fi
  cut -c1-300 ${O}_blockers.jsonl ;;
pmc)
  SETS=${COUNTER_SETS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT;SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"}
  IFS=';' read -ra CS <<< "$SETS"; i=0
  for set in "${CS[@]}"; do
    i=$((i + 1)); rm -rf /tmp/plx_pmc
    timeout -s KILL ${LIMIT:-150} rocprofv3 --pmc $set -d /tmp/plx_pmc -o run --output-format csv -- "$@" \
      > ${O}_pmc$i.log 2>&1 || fail "pmc pass $i" $? ${O}_pmc$i.log
    f=$(find /tmp/plx_pmc -name '*counter_collection.csv' | head -1)
    python3 scripts/pmc_summary.py "$f" ${MATCH:+--match $MATCH} > ${O}_pmc$i.jsonl
    cut -c1-700 ${O}_pmc$i.jsonl
  done ;;
py)
  timeout -k 10 ${LIMIT:-600} python -u "$@" > $O.out 2> $O.err || fail "$1" $? $O.err
  tail -${SHOW:-20} $O.out ;;
suite)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 120 --timeout-method thread \
    > ${O}_gp.log 2>&1 || fail "GP tests" $? ${O}_gp.log
  timeout -k 10 900 python scripts/bench_suite.py --only ${SUITE:-iris,hb_reduce,bo,mlp_grid,lm_gpt2,lm_llama8b} \
    --bo-backends hip ${SUITE_ARGS:-} > $O.jsonl 2> $O.err || fail suite $? $O.err
  cat $O.jsonl ;;
*)
  echo "unknown mode '$MODE' (see the header of scripts/gpu.sh)"; exit 2 ;;
esac
