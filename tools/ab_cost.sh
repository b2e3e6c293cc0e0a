#!/bin/bash
# Interleaved A/B of the OpenCV-mode cost stage: the two-kernel form (SGM_OCV_FUSED=0) against
# the fused kernel at each disparity-pair width (SGM_FUSE_DPC) or band height (SGM_FUSE_ROWS), per
# case of ocv_modes_bench.py. Build-time knobs (SGM_FUSE_RING8, _BOX_EARLY, _NB_WIDE, _WPE): variant
# libraries from tools/build_variant.sh, timed with tools/ab_ocv.sh.
# Usage: tools/ab_cost.sh <rounds> <case filter> [variants...]; lines to gpurun_out/ab_cost.jsonl
set -u
rounds=${1:-2}; case=${2:-}; shift 2 || true
variants=${*:-"unfused fused fused16 fused8"}
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for v in $variants; do
    case $v in
      unfused) env=(SGM_OCV_FUSED=0) ;;
      fused) env=(SGM_OCV_FUSED=1) ;;
      fused32) env=(SGM_OCV_FUSED=1 SGM_FUSE_DPC=32) ;;
      fused16) env=(SGM_OCV_FUSED=1 SGM_FUSE_DPC=16) ;;
      fused8) env=(SGM_OCV_FUSED=1 SGM_FUSE_DPC=8) ;;
      fused_rows*) env=(SGM_OCV_FUSED=1 SGM_FUSE_ROWS=${v#fused_rows}) ;;
    esac
    env "${env[@]}" timeout -k 10 300 python tools/ocv_modes_bench.py --reps 5 --case "$case" > gpurun_out/ab_cost_one.log 2>&1 || exit 1
    python3 - "$v" "$r" <<'PY' >> gpurun_out/ab_cost.jsonl
import json, sys
for l in open("gpurun_out/ab_cost_one.log"):
    if l.startswith("{"):
        d = json.loads(l)
        st = {s["name"]: s["avg_ms"] for s in d["stages"]}
        print(json.dumps({"variant": sys.argv[1], "round": int(sys.argv[2]), "case": d["case"],
                          "ms_per_frame": d["gpu_ms_per_frame"], "cost_ms": st.get("ocv_cost")}))
PY
  done
done
