#!/bin/bash
# GPU box: the OpenCV-mode path launch's cache behaviour on one box: the box's measured
# HBM copy rate, then per case one line of tools/ocv_modes_bench.py and PMC passes (L2 hits / misses,
# FETCH_SIZE, WRITE_SIZE, VALU) summarised per kernel by tools/ocv_pmc_summary.py.
#   bash tools/ocv_paths_cache.sh TAG ["case|case"]
set -u
export TMPDIR=/tmp
TAG=${1:-paths_cache}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python3 -c "import bench, torch; torch.cuda.set_device(0); print('copy_GBps', bench.hbm_copy_gbps(0))" \
    > $O/copy_rate.txt 2>&1 || exit 1
IFS='|' read -r -a CASE_LIST <<< "${2:-refcfg 2448x2048 minD 147 D 480 block 21 MODE_SGBM (gated)|1920x1080 D=128 MODE_SGBM}"
for c in "${CASE_LIST[@]}"; do
  n=$(echo "$c" | tr -dc 'A-Za-z0-9' | cut -c1-40)
  timeout -k 10 300 python3 tools/ocv_modes_bench.py --reps 10 --case "$c" > $O/line_$n.log 2>&1 || exit 1
  i=0
  for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc_$n -o pass$i --output-format csv -- \
        python3 tools/ocv_modes_bench.py --reps 2 --case "$c" > $O/pmc_${n}_$i.log 2>&1 || exit 1
  done
  python3 tools/ocv_pmc_summary.py $O/pmc_$n > $O/summary_$n.txt || exit 1
  find $O/pmc_$n -mindepth 1 -type d -exec rm -rf {} +
done
cat $O/copy_rate.txt $O/summary_*.txt
