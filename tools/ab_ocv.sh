#!/bin/bash
# GPU box: interleaved A/B of the OpenCV-mode timings (tools/ocv_modes_bench.py). A variant is
# a library built by tools/build_variant.sh (SGM_HIP_LIB), "base" (the in-tree one) or an
# environment assignment NAME=VALUE run with the in-tree library, or VARIANT+NAME=VALUE (both).
#   bash tools/ab_ocv.sh CASE_SUBSTRING ROUNDS variant1 variant2 ...
set -u
CASE=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=""; envv=""
    case $v in
      base) ;;
      base+*=*) envv=${v#*+} ;;
      *+*=*) lib=i3dr_stereo_camera-ros_amd/lib/variants/${v%%+*}/libsgm_hip.so; envv=${v#*+} ;;
      *=*) envv=$v ;;
      *) lib=i3dr_stereo_camera-ros_amd/lib/variants/$v/libsgm_hip.so ;;
    esac
    env $envv SGM_HIP_LIB=$lib timeout -k 10 300 python tools/ocv_modes_bench.py --reps 5 --case "$CASE" 2>/dev/null \
      | grep '^{' | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ab_ocv.jsonl || exit 1
  done
done
