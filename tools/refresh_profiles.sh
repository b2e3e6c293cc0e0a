#!/bin/bash
# GPU box: one consistent refresh of the measurement files of a round, from the build in the
# tree. For C3 and C2: PMC passes (tools/pmc.sh) -> <cfg>_pmc.json, the bench line (the
# default bench run; C3 with its cpu_baseline), and a rocprofv3 --kernel-trace --stats run of
# the bench whose per-launch durations are set beside its HIP-event stage times
# (tools/prof_compare.py). Everything lands in gpurun_out/<TAG>/; copy into profiles/.
#   bash tools/refresh_profiles.sh TAG GIT_REV
set -u
export TMPDIR=/tmp
TAG=${1:-latest}
REV=${2:-unknown}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step NAME SECONDS CMD... (stdout+stderr -> $O/NAME.log); any failure ends the script
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc != 0 ]; then tail -n 8 "$O/$name.log"; exit $rc; fi
}
for cfg in c3 c2; do
  step ${cfg}_pmc 900 env PMC_DIR=$O/pmc_$cfg BENCH_ARGS="--config $cfg" bash tools/pmc.sh
  python3 tools/pmc_summary.py $O/pmc_$cfg --config $cfg --git "$REV" --out $O/${cfg}_pmc.json > /dev/null || exit 1
  cp $O/${cfg}_pmc.json profiles/latest_pmc_${cfg}.json     # bench.py quotes it as traffic_profile
  rm -rf $O/pmc_$cfg/*/                                     # per-agent raw dirs (large)
done
step c3_bench 600 python3 bench.py
step c2_bench 600 python3 bench.py --config c2 --no-cpu-baseline
for cfg in c3 c2; do
  rm -rf $O/prof_$cfg
  step ${cfg}_rocprof 600 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-c5
  python3 tools/prof_compare.py "$(find $O/prof_$cfg -name '*kernel_trace.csv' | head -1)" \
      $O/${cfg}_rocprof.log > $O/${cfg}_prof_vs_bench.txt || exit 1
  cp "$(find $O/prof_$cfg -name '*kernel_stats.csv' | head -1)" $O/${cfg}_kernel_stats.csv
  rm -rf $O/prof_$cfg
done
echo done
