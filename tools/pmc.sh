#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel-trace only).
#   PMC_DIR (default gpurun_out/pmc), BENCH_ARGS (e.g. "--config c2")
# 32 frames = 16 two-frame groups: the largest-grid fused launches are then 14 steady-state
# launches and the pipeline's first one.
set -u
D=${PMC_DIR:-gpurun_out/pmc}
mkdir -p $D
export TMPDIR=/tmp
CMD="python3 bench.py --steps 1 --warmup 1 --frames 32 --no-cpu-baseline --no-c5 ${BENCH_ARGS:-}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp -d $D -o pass$i --output-format csv -- $CMD > $D/pass$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 $D/pass$i.log
  case $rc in 0) ;; *) echo "pass $i failed: stopping"; exit $rc;; esac
done
