#!/bin/bash
set -u
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
for k in 2 4; do
  for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    tag=$(echo $grp | cut -c1-8)
    SGM_PERSIST=$k timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc3 -o k${k}_$tag --output-format csv -- python3 bench.py --steps 2 --warmup 1 --frames 2 --no-cpu-baseline --no-pipeline > gpurun_out/pmc3/k${k}_$tag.log 2>&1
    rc=$?; echo "k=$k $tag rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
