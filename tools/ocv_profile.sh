#!/bin/bash
# GPU box: OCV-mode (the reference's own matcher) measurement files of a round:
# tools/ocv_modes_bench.py lines (CPU restatement beside for the small cases), a rocprofv3
# kernel trace + stats of the C1 and 1080p cases, and PMC (FETCH/WRITE/VALU) of the same.
#   bash tools/ocv_profile.sh TAG
#   CASES="D 752 block 21 MODE_SGBM|D 752 block 21 MODE_HH" MODES=0 bash tools/ocv_profile.sh TAG
# (CASES: '|'-separated case-name substrings to trace and count; MODES=0 skips the full modes run)
set -u
export TMPDIR=/tmp
TAG=${1:-latest}
O=gpurun_out/$TAG
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc != 0 ]; then tail -n 8 "$O/$name.log"; exit $rc; fi
}
if [ "${MODES:-1}" != 0 ]; then
  step ocv_modes 900 python3 tools/ocv_modes_bench.py --reps 10 --cpu
  grep '^{' $O/ocv_modes.log > $O/ocv_modes.jsonl
fi
IFS='|' read -r -a CASE_LIST <<< "${CASES:-C1|1920x1080}"
for c in "${CASE_LIST[@]}"; do
  n=$(echo "$c" | tr -dc 'A-Za-z0-9')
  rm -rf $O/prof_$n
  step ocv_rocprof_$n 600 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- \
      python3 tools/ocv_modes_bench.py --reps 10 --case "$c"
  cp "$(find $O/prof_$n -name '*kernel_stats.csv' | head -1)" $O/ocv_${n}_kernel_stats.csv
  cp "$(find $O/prof_$n -name '*kernel_trace.csv' | head -1)" $O/ocv_${n}_kernel_trace.csv
  rm -rf $O/prof_$n
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    step ocv_pmc_${n}_$i 300 rocprofv3 --pmc $grp -d $O/pmc_$n -o pass$i --output-format csv -- \
        python3 tools/ocv_modes_bench.py --reps 2 --case "$c"
  done
  python3 tools/ocv_pmc_summary.py $O/pmc_$n > $O/ocv_${n}_pmc.txt
  find $O/pmc_$n -mindepth 1 -type d -exec rm -rf {} +
done
echo done
