set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --no-cpu-baseline --host-io > gpurun_out/b_host.log 2>&1 || { tail -20 gpurun_out/b_host.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/b_dev.log 2>&1 || { tail -20 gpurun_out/b_dev.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/b_dev.log gpurun_out/b_host.log
