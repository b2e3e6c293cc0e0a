#!/bin/bash
# Build an A/B variant of libsgm_hip.so with extra -D flags on some sources (default
# census_sgm.hip; several: "census_sgm.hip sgm_api.cpp"), the other objects reused from the
# in-tree build; load it with SGM_HIP_LIB=i3dr_stereo_camera-ros_amd/lib/variants/NAME/libsgm_hip.so.
#   bash tools/build_variant.sh NAME "-DSGM_X=1 -DSGM_Y=2" ["source.hip other.cpp"]
set -eu
NAME=$1; DEFS=$2; SRCS=${3:-census_sgm.hip}
P=i3dr_stereo_camera-ros_amd
OUT=$P/lib/variants/$NAME
mkdir -p $OUT
python3 -c "import __graft_entry__ as g; g.build()" > /dev/null
objs=""
for o in $P/lib/obj/*.o; do
  b=$(basename $o .o)
  if [[ " $SRCS " == *" $b "* ]]; then
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I$P/csrc -Iinclude -Wno-unused-function $DEFS \
        -x hip -c $P/csrc/$b -o $OUT/$b.o
    objs="$objs $OUT/$b.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsgm_hip.so $objs -lpthread
echo "built $OUT/libsgm_hip.so ($DEFS)"
