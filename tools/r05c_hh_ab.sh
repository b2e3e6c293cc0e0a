#!/bin/bash
# round-5 GPU step: 1080p MODE_HH with and without the fused vertical WTA now that the row WTA is
# packed (the unfused frame takes deficit volumes and k_ocv_wta16_pk)
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_ocv.jsonl
timeout -k 10 600 bash tools/ab_ocv.sh "1920x1080 D=128 MODE_HH" 3 base base+SGM_OCV_VWTA=0 || exit 1
cp gpurun_out/ab_ocv.jsonl gpurun_out/r05c_hh_vwta_ab.jsonl
