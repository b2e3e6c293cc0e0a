#!/bin/bash
# GPU box: PMC passes -> profiles/latest_pmc.json, then smoke + GPU tests + bench + rocprofv3
# kernel trace (the bench's roofline.traffic reads the fresh PMC summary). Results under
# gpurun_out/; copy the ones to keep into profiles/ afterwards.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc --out profiles/latest_pmc.json > gpurun_out/pmc_summary.txt 2>&1 || exit 1
cp profiles/latest_pmc.json gpurun_out/latest_pmc.json
bash tools/gpu_check.sh all
