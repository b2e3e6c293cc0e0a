#!/bin/bash
# round-5 GPU step: HBM bytes of the 1080p OpenCV-mode path launch with the directions' blocks dealt
# in turn (SGM_OCV_ILV=1) or one direction after another (0): FETCH_SIZE / WRITE_SIZE / VALU passes,
# summarised by tools/ocv_pmc_summary.py
set -u
mkdir -p gpurun_out/r05c_ilv
export TMPDIR=/tmp
for ilv in 0 1; do
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    n=$(echo $grp | cut -d' ' -f1)
    SGM_OCV_ILV=$ilv timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/r05c_ilv/pmc_$ilv -o pass_$n --output-format csv -- \
        python3 tools/ocv_modes_bench.py --reps 2 --case "1920x1080 D=128 MODE_SGBM" > gpurun_out/r05c_ilv/${ilv}_$n.log 2>&1 || exit 1
  done
  python3 tools/ocv_pmc_summary.py gpurun_out/r05c_ilv/pmc_$ilv > gpurun_out/r05c_ilv/summary_$ilv.txt || exit 1
done
echo ilv-pmc-done
