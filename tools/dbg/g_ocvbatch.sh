set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ocv.py -k "batch_lanes" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ob.log 2>&1 || { tail -30 gpurun_out/t_ob.log; exit 1; }
tail -2 gpurun_out/t_ob.log
timeout -k 10 600 python3 tools/dbg/ocv_batch_bench.py
