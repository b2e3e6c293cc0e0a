#!/bin/bash
# GPU-box driver: smoke -> GPU tests -> short bench. Each GPU step has its own time limit;
# any crash-class exit (timeout 124/137, abort 134, segfault 139) ends the script at once.
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
MODE=${1:-all}   # all | tests | bench | prof | ocv | trace | ab <configs> <rounds> <variants...>
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || { [ "$MODE" = all ] || exit 1; }
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  run gpu_tests 1200 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  run bench 600 python bench.py --steps 5 --warmup 2
fi
if [ "$MODE" = ocv ]; then        # OpenCV modes: their GPU tests, per-stage lines, host calls
  run gpu_tests_ocv 600 python -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_refcfg.py \
      tests/test_gpu_ocv_vwta.py -q -x --timeout=300 -p no:cacheprovider || exit 1
  run ocv_modes 600 python tools/ocv_modes_bench.py --reps 10 || exit 1
  run host_calls 300 python tools/host_calls.py || exit 1
fi
if [ "$MODE" = trace ]; then      # SGM_TRACE timelines of the single-frame paths launch
  SGM_TRACE=/tmp/tr_c5.bin run trace_c5 120 python tools/trace_single.py --config c5 || exit 1
  SGM_TRACE=/tmp/tr_c2.bin run trace_c2 120 python tools/trace_single.py --config c2 || exit 1
fi
if [ "$MODE" = ab ]; then         # interleaved single-frame A/B of variant builds: ab <configs> <rounds> <variants...>
  shift
  bash tools/ab_single.sh "$@" || exit 1
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  rm -rf gpurun_out/prof
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  python3 tools/prof_compare.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/rocprof.log > gpurun_out/prof_vs_bench.txt
fi
exit 0
