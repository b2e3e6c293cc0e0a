#!/bin/bash
# round-5 GPU step: 12 MP OpenCV-mode frames with D <= 256, fused vertical WTA against the packed
# row WTA (SGM_OCV_VWTA=1 / 0), interleaved
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 900 bash tools/ab_ocv.sh "12MP" 2 base+SGM_OCV_VWTA=1 base+SGM_OCV_VWTA=0 || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_12mp_ab.jsonl
