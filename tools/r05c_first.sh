set -u
bash tools/gpu_check.sh tests || exit 1
cp gpurun_out/gpu_tests.log gpurun_out/r05c_gpu_full.log
timeout -k 10 400 bash tools/ocv_cost_pmc.sh r05c_pmc1080 "1920x1080 D=128 MODE_SGBM" || exit 1
