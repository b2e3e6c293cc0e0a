set -u
mkdir -p gpurun_out
SGM_GROUP=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_census.py -k "device_batch_pipeline" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_g3.log 2>&1; tail -15 gpurun_out/t_g3.log
SGM_GROUP=3 SGM_TRACE=gpurun_out/g3tr.%d timeout -k 10 300 python3 tools/dbg/trace_upwta.py 2>&1 | tail -20
rm -f gpurun_out/g3tr.*
