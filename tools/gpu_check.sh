#!/bin/bash
# GPU-box driver: every GPU step of a round goes through this script. Each GPU step has its own
# time limit; any crash-class exit (timeout 124/137, abort 134, segfault 139) ends the script at
# once. Logs: gpurun_out/<name>.log. Modes:
#   all | tests | bench | prof          smoke, the full GPU suite, a short bench, rocprofv3 of it
#   final                               smoke, the full GPU suite, the default bench line
#   parity <test files...>              those GPU test files (e.g. the OpenCV-mode set after a change)
#   fuzz <cases> [k-expr]               tests/test_gpu_fuzz.py at SGM_FUZZ_CASES=<cases> (env passes through,
#                                       e.g. SGM_OCV_FUSED=1 bash tools/gpu_check.sh fuzz 3000 ocv)
#   ocv                                 the OpenCV-mode tests, every ocv_modes_bench line, host calls
#   ocvlines                            every ocv_modes_bench line (no CPU restatement)
#   abocv "<case>" <rounds> <variants>  interleaved OpenCV-mode A/B (tools/ab_ocv.sh)
#   ab <configs> <rounds> <variants>    interleaved single-frame census A/B (tools/ab_single.sh)
#   trace                               SGM_TRACE timelines of the single-frame paths launch
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if crash $rc; then echo "CRASH-CLASS EXIT in $name: stopping"; exit $rc; fi
  return $rc
}
PYTEST="python -u -m pytest -m gpu -x -q --timeout-method thread -p no:cacheprovider"
MODE=${1:-all}
shift || true
case $MODE in
  parity)
    run parity 1100 $PYTEST --timeout 900 "$@"; exit $? ;;
  fuzz)
    N=$1; K=${2:-}
    run fuzz$N 1100 env SGM_FUZZ_CASES=$N $PYTEST --timeout 1000 ${K:+-k "$K"} tests/test_gpu_fuzz.py; exit $? ;;
  ocvlines)
    run ocv_lines 900 python tools/ocv_modes_bench.py --reps 10 || exit 1
    grep '^{' gpurun_out/ocv_lines.log > gpurun_out/ocv_lines.jsonl; exit 0 ;;
  abocv)
    rm -f gpurun_out/ab_ocv.jsonl
    run abocv 1100 bash tools/ab_ocv.sh "$@"; exit $? ;;
  ab)
    bash tools/ab_single.sh "$@" || exit 1; exit 0 ;;
  trace)
    SGM_TRACE=/tmp/tr_c5.bin run trace_c5 120 python tools/trace_single.py --config c5 || exit 1
    SGM_TRACE=/tmp/tr_c2.bin run trace_c2 120 python tools/trace_single.py --config c2 || exit 1
    exit 0 ;;
esac
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || { [ "$MODE" = all ] || exit 1; }
if [ "$MODE" = all ] || [ "$MODE" = tests ] || [ "$MODE" = final ]; then
  run gpu_tests 1200 $PYTEST --timeout 900 tests || exit 1
fi
if [ "$MODE" = final ]; then
  run bench_final 600 python bench.py || exit 1
  grep '^{' gpurun_out/bench_final.log > gpurun_out/bench_final.json
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  run bench 600 python bench.py --steps 5 --warmup 2
fi
if [ "$MODE" = ocv ]; then        # OpenCV modes: their GPU tests, per-stage lines, host calls
  run gpu_tests_ocv 900 $PYTEST --timeout 600 tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py \
      tests/test_gpu_refcfg.py tests/test_gpu_ocv_vwta.py || exit 1
  run ocv_modes 600 python tools/ocv_modes_bench.py --reps 10 || exit 1
  run host_calls 300 python tools/host_calls.py || exit 1
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  rm -rf gpurun_out/prof
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  python3 tools/prof_compare.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/rocprof.log > gpurun_out/prof_vs_bench.txt
fi
exit 0
