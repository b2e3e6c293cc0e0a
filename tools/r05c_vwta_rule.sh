#!/bin/bash
# round-5 GPU step: OCV parity after the row-WTA / fused-vertical-WTA rule change (D <= 128: row)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_ocv_vwta.py \
    tests/test_gpu_ocv_evol.py tests/test_gpu_ocv_wta_pk.py tests/test_gpu_refcfg.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_vwta_rule_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_vwta_rule_tests.log; exit $rc
