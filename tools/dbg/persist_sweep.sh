set -u
timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/t.log 2>&1 || { tail -5 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for k in 2 3 4 6; do
  SGM_PERSIST=$k timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_$k.log 2>&1 || exit $?
  SGM_PRIO=1 SGM_PERSIST=$k timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_p$k.log 2>&1 || exit $?
done
SGM_PERSIST=4 SGM_TRACE=gpurun_out/trace_4.bin timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr_4.log 2>&1
