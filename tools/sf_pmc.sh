#!/bin/bash
# PMC passes over single-frame calls (tools/single_frame.py; one counter group per pass,
# kernel-trace only): per-kernel VALU / busy / HBM bytes of the paths and WTA launches.
#   bash tools/sf_pmc.sh CONFIG [DIR]     e.g. c5 -> gpurun_out/sfpmc_c5
set -u
CF=${1:-c5}
D=${2:-gpurun_out/sfpmc_$CF}
mkdir -p $D
export TMPDIR=/tmp
CMD="python3 tools/single_frame.py --configs $CF --reps 3"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp -d $D -o pass$i --output-format csv -- $CMD > $D/pass$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 $D/pass$i.log
  case $rc in 0) ;; *) echo "pass $i failed: stopping"; exit $rc;; esac
done
