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
MODE=${1:-all}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || { [ "$MODE" = all ] || exit 1; }
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  run gpu_tests 1200 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  run bench 600 python bench.py --steps 5 --warmup 2
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  rm -rf gpurun_out/prof
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  python3 tools/prof_compare.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/rocprof.log > gpurun_out/prof_vs_bench.txt
fi
exit 0
