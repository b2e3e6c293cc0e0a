#!/bin/bash
# GPU box: rocprofv3 kernel trace of single-frame calls (tools/single_frame.py) -> per-kernel
# durations, launch gaps and a compact trace under gpurun_out/.
#   bash tools/sf_profile.sh [configs] [reps]
set -u
export TMPDIR=/tmp
CF=${1:-c2,c3,c5}
REPS=${2:-10}
mkdir -p gpurun_out
rm -rf gpurun_out/sf
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sf -o run --output-format csv -- \
    python3 tools/single_frame.py --configs "$CF" --reps "$REPS" > gpurun_out/sf.log 2>&1 || exit $?
f=$(find gpurun_out/sf -name "*kernel_trace.csv" | head -1)
cp "$(find gpurun_out/sf -name '*kernel_stats.csv' | head -1)" gpurun_out/sf_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
with open("gpurun_out/sf_trace_small.csv", "w") as o:
    for r in rows:
        o.write("%s,%d,%d,%s\n" % (r["Kernel_Name"].split("(")[0][-60:], int(r["Start_Timestamp"]),
                                   int(r["End_Timestamp"]), r["Grid_Size_X"]))
PY
rm -rf gpurun_out/sf
