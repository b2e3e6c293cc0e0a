#!/bin/bash
# round-5 GPU step: smoke + the full GPU suite at the current build
set -u
bash tools/gpu_check.sh tests || exit 1
cp gpurun_out/gpu_tests.log gpurun_out/r05c_gpu_full2.log
