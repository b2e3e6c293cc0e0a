#!/bin/bash
# round-5 GPU step: fused-cost box variants (window as dwords, branch-free descriptor stores):
# parity of the default build, then an interleaved A/B against the previous build (pf)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ocv_fused.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r05c_box_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_box_tests.log; [ $rc = 0 ] || exit $rc
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 600 bash tools/ab_ocv.sh "1920x1080 D=128 MODE_SGBM" 3 pf base nb w32 w32nb || exit 1
timeout -k 10 600 bash tools/ab_ocv.sh "MODE_SGBM (gated)" 2 pf base nb w32 w32nb || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_box_ab.jsonl
