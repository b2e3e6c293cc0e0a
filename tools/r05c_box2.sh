#!/bin/bash
# round-5 GPU step: the branch-free box stores for R <= 9 (default build) and the descriptor stores
# for wider boxes (variant bufw): OCV parity of the default build, then an interleaved A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ocv.py tests/test_gpu_ocv_compat.py tests/test_gpu_ocv_fused.py \
    tests/test_gpu_refcfg.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05c_box2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_box2_tests.log; [ $rc = 0 ] || exit $rc
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 600 bash tools/ab_ocv.sh "1920x1080 D=128 MODE_SGBM" 3 pf base || exit 1
timeout -k 10 600 bash tools/ab_ocv.sh "MODE_SGBM (gated)" 3 pf base bufw || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_box2_ab.jsonl
