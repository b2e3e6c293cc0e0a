mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_refcfg.py -q -x --timeout=300 -p no:cacheprovider > gpurun_out/gpu_tests_ocv.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_ocv.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/ocv_modes_bench.py --reps 10 --case MODE_SGBM > gpurun_out/ocv_modes.log 2>&1 || exit $?
SGM_OCV_ROWS=0 timeout -k 10 600 python tools/ocv_modes_bench.py --reps 10 --case MODE_SGBM > gpurun_out/ocv_modes0.log 2>&1 || exit $?
timeout -k 10 300 python tools/host_calls.py > gpurun_out/host_calls.log 2>&1 || exit $?
SGM_HOST_CHUNKS=0 timeout -k 10 300 python tools/host_calls.py > gpurun_out/host_calls0.log 2>&1
