#!/bin/bash
# round-5 GPU step: OCV parity with the 4-pixel prefilter, then an interleaved A/B against the
# previous build (variant head0)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_ocv_fused.py \
    tests/test_gpu_ocv_evol.py tests/test_gpu_ocv_wta_pk.py tests/test_gpu_refcfg.py \
    -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_prefilter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_prefilter_tests.log; [ $rc = 0 ] || exit $rc
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 600 bash tools/ab_ocv.sh "1920x1080" 3 base head0 || exit 1
timeout -k 10 600 bash tools/ab_ocv.sh "gated" 2 base head0 || exit 1
timeout -k 10 300 bash tools/ab_ocv.sh "C1" 3 base head0 || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_prefilter_ab.jsonl
