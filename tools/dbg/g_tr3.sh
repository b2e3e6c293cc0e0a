# single-frame traces of timing-only variants (SGM_EXP 8: aligned diagonal segment loads,
# 16: diagonal stores at the vertical addresses); per-direction us/step
set -u
mkdir -p gpurun_out/tr3
for v in base e8 e16; do
  lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
  [ $v != base ] && lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so
  SGM_HIP_LIB=$lib TRACE_D=128 SGM_TRACE=gpurun_out/tr3/$v.%d timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr3_$v.log 2>&1 || { tail gpurun_out/tr3_$v.log; exit 1; }
  python tools/dbg/trace_analyze.py gpurun_out/tr3/$v.1
done
