# priority build checks: census tests, single/batch timing, OCV variants (base / op / op4)
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_census.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_census.log 2>&1 || { tail -20 gpurun_out/t_census.log; exit 1; }
tail -1 gpurun_out/t_census.log
LIBS=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so CASES=1080x1920x128,1080x1920x256,3000x4096x512 NF=4 ROUNDS=1 timeout -k 10 300 python3 tools/dbg/lib_ab.py || exit 1
VARIANTS="base op op4" CASE="" bash tools/dbg/g_ocv_var.sh
