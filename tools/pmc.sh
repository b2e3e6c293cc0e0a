#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel-trace only).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --frames 8 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc -o pass$i --output-format csv -- $CMD > gpurun_out/pmc/pass$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 gpurun_out/pmc/pass$i.log
  case $rc in 124|134|137|139) echo "crash-class exit: stopping"; exit $rc;; esac
done
