set -u
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
SGM_TRACE=gpurun_out/tr/base.%d timeout -k 10 300 python tools/dbg/trace_upwta.py > gpurun_out/tr_base.txt 2>&1 || { tail gpurun_out/tr_base.txt; exit 1; }
SGM_HIP_LIB=i3dr_stereo_camera-ros_amd/lib/variants/lib_prio1.so SGM_TRACE=gpurun_out/tr/p1.%d timeout -k 10 300 python tools/dbg/trace_upwta.py > gpurun_out/tr_p1.txt 2>&1 || exit 1
cat gpurun_out/tr_base.txt gpurun_out/tr_p1.txt
rm -rf gpurun_out/tr
ROUNDS=2 bash tools/dbg/variants.sh prio1 prio3
