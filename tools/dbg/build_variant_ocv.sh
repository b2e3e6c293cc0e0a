#!/bin/bash
# build_variant_ocv.sh NAME "EXTRA HIPCC FLAGS" — libsgm_hip.so with ocv_sgm.hip compiled under
# extra flags, into lib/variants/lib_NAME.so (use with SGM_HIP_LIB=...)
set -eu
cd "$(dirname "$0")/../.."
P=i3dr_stereo_camera-ros_amd
mkdir -p $P/lib/variants
python -c "import sys; sys.path.insert(0,'$P'); import build_ext; build_ext.build(verbose=False)"
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I$P/csrc -Iinclude $2 -x hip -c $P/csrc/ocv_sgm.hip -o /tmp/ocv_$1.o
objs=$(ls $P/lib/obj/*.o | grep -v ocv_sgm)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/lib_$1.so /tmp/ocv_$1.o $objs -lpthread
echo built $P/lib/variants/lib_$1.so
