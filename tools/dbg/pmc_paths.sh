#!/bin/bash
# Stall-analysis PMC passes on the standalone path kernel (bench --no-pipeline).
set -u
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --frames 2 --no-cpu-baseline --no-pipeline"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc2 -o pass$i --output-format csv -- $CMD > gpurun_out/pmc2/pass$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  case $rc in 124|134|137|139) echo "crash-class exit: stopping"; exit $rc;; esac
done
