mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/ocv_modes_bench.py --reps 10 > gpurun_out/ocv_modes.log 2>&1 || exit $?
timeout -k 10 300 python tools/host_calls.py > gpurun_out/host_calls.log 2>&1 || exit $?
SGM_TRACE=/tmp/tr.bin timeout -k 10 120 python tools/trace_single.py --config c5 > gpurun_out/trace_c5.txt 2>&1 || exit $?
SGM_TRACE=/tmp/tr2.bin timeout -k 10 120 python tools/trace_single.py --config c2 > gpurun_out/trace_c2.txt 2>&1
