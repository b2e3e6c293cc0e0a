# correctness (gpu tests) then C3 bench pipelined + unpipelined
set -u
timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/t.log 2>&1 || { tail -8 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/b2.log 2>&1 || exit $?
