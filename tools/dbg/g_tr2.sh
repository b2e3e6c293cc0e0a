# single-frame trace + A/B: base vs trash-spread variant (SGM_VOL_PAD makes room for the slots)
set -u
mkdir -p gpurun_out/tr2
export SGM_VOL_PAD=262144
for v in base ts; do
  lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
  [ $v = ts ] && lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_ts.so
  SGM_HIP_LIB=$lib TRACE_D=128 SGM_TRACE=gpurun_out/tr2/$v.%d timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr2_$v.log 2>&1 || { tail gpurun_out/tr2_$v.log; exit 1; }
  python tools/dbg/trace_analyze.py gpurun_out/tr2/$v.1
done
rm -rf gpurun_out/tr2
LIBS=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so,i3dr_stereo_camera-ros_amd/lib/variants/lib_ts.so CASES=1080x1920x128,1080x1920x256 ROUNDS=2 timeout -k 10 300 python3 tools/dbg/lib_ab.py
