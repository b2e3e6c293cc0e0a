#!/bin/bash
# GPU box: PMC of the DESIGN §8.2 prototype A/B (tools/strip3_ab.py, experiment build): VALU
# instructions, LDS instructions and HBM bytes per launch of k_strip3_proto and of the production
# k_census_paths16 launches (three top-down directions; all eight), per config. One counter
# group per pass. Summary: gpurun_out/strip3_pmc/summary.txt (per kernel and grid size).
set -u
export TMPDIR=/tmp
O=gpurun_out/strip3_pmc
mkdir -p $O
export SGM_HIP_LIB=i3dr_stereo_camera-ros_amd/lib/variants/strip3/libsgm_hip.so
CMD="python3 tools/strip3_ab.py --reps 2 --rounds 1 --shapes 32:8"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $grp ($(date +%T))"
  timeout -s KILL 180 rocprofv3 --pmc $grp -d $O/pmc -o pass$i --output-format csv -- $CMD > $O/pass$i.log 2>&1 \
    || { tail -5 $O/pass$i.log; exit 1; }
done
python3 - $O/pmc > $O/summary.txt <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/pass*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "paths16" not in k and "strip3" not in k:
            continue
        acc[(k, r.get("Grid_Size", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, gs), cs in sorted(acc.items()):
    print(f"{k}  grid {gs}")
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
find $O/pmc -mindepth 1 -type d -exec rm -rf {} +
cat $O/summary.txt
