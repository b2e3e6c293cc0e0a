#!/bin/bash
# GPU box: interleaved A/B of single-frame latency (tools/single_frame.py) between the in-tree
# library and variants built by tools/build_variant.sh.
#   bash tools/ab_single.sh "c2,c3" ROUNDS variant1 variant2 ...
set -u
CF=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib=i3dr_stereo_camera-ros_amd/lib/variants/$v/libsgm_hip.so; fi
    SGM_HIP_LIB=$lib timeout -k 10 300 python tools/single_frame.py --configs $CF --reps 30 2>/dev/null \
      | grep '^{' | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ab_single.jsonl || exit 1
  done
done
