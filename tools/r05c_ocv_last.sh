#!/bin/bash
# round-5 GPU step: the OpenCV-mode lines at the final build (every case, no CPU restatement)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python tools/ocv_modes_bench.py --reps 10 > gpurun_out/r05c_ocv_last.log 2>&1 || exit 1
grep '^{' gpurun_out/r05c_ocv_last.log > gpurun_out/r05c_ocv_modes_last.jsonl
