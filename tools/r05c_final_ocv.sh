#!/bin/bash
# round-5 GPU step (final OCV refresh at the session's last kernel build): a 3000-case fuzz of every
# entry point, the OpenCV-mode lines / rocprofv3 stats / PMC (tools/ocv_profile.sh), and the PMC of
# every OCV kernel on the shipped 2448x2048 D=480 block-21 MODE_SGBM frame
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SGM_FUZZ_CASES=3000 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r05c_fuzz3000.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_fuzz3000.log; [ $rc = 0 ] || exit $rc
bash tools/ocv_profile.sh r05c || exit 1
timeout -k 10 400 bash tools/ocv_cost_pmc.sh r05c_refcfg "refcfg 2448x2048 minD 147 D 480 block 21 MODE_SGBM (gated)" \
    > /dev/null || exit 1
echo final-ocv-done
