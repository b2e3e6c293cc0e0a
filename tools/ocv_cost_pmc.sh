#!/bin/bash
# GPU box: stall / LDS / HBM counters of the OpenCV-mode cost kernels on one case, fused or not:
#   SGM_OCV_FUSED=1 bash tools/ocv_cost_pmc.sh TAG "refcfg 2448x2048 minD 147 D 480 block 21 MODE_SGBM (gated)"
# Per-kernel averages (one line per kernel and counter) to gpurun_out/TAG/cost_pmc.txt.
set -u
export TMPDIR=/tmp
TAG=${1:-cost_pmc}
CASE=${2:-1920x1080 D=128 MODE_SGBM}
O=gpurun_out/$TAG
mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $grp ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc -o pass$i --output-format csv -- \
      python3 tools/ocv_modes_bench.py --reps 2 --case "$CASE" > $O/pass$i.log 2>&1 || { tail -5 $O/pass$i.log; exit 1; }
done
python3 - $O/pmc > $O/cost_pmc.txt <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/pass*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "ocv" not in k:
        continue
    print(k)
    for c in sorted(cs):
        print(f"   {c:24s} {sum(cs[c]) / len(cs[c]):16.1f}  (n={len(cs[c])})")
PY
find $O/pmc -mindepth 1 -type d -exec rm -rf {} +
cat $O/cost_pmc.txt
