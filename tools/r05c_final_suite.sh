#!/bin/bash
# round-5 GPU step at the session's last build: smoke + the full GPU suite, then a 12000-case fuzz
# of every entry point and a 3000-case fuzz with the fused OCV cost forced on small frames
set -u
bash tools/gpu_check.sh tests || exit 1
cp gpurun_out/gpu_tests.log gpurun_out/r05c_gpu_full_final.log
export TMPDIR=/tmp
SGM_FUZZ_CASES=12000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 800 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_fuzz12000.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_fuzz12000.log; [ $rc = 0 ] || exit $rc
SGM_OCV_FUSED=1 SGM_FUZZ_CASES=3000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -k ocv \
    --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_fuzz3000_fused.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_fuzz3000_fused.log; exit $rc
