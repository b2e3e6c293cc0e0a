#!/bin/bash
# round-5 GPU step: k_ocv_paths with the block's direction / slot stated uniform (no waterfall around
# the buffer ops of the small-D instantiations): OCV parity, then an interleaved A/B against the
# previous build (variant pre)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_ocv_evol.py \
    tests/test_gpu_ocv_wta_pk.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r05c_uniform_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_uniform_tests.log; [ $rc = 0 ] || exit $rc
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 300 bash tools/ab_ocv.sh "C1" 3 pre base || exit 1
timeout -k 10 600 bash tools/ab_ocv.sh "1920x1080 D=128 MODE_SGBM" 2 pre base || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_uniform_ab.jsonl
