set -u
timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/t.log 2>&1 || { tail -8 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for G in 1 2 3 4; do
  SGM_GROUP=$G timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_g$G.log 2>&1 || exit $?
done
SGM_GROUP=2 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --frames 16 --no-cpu-baseline > gpurun_out/b_g2f16.log 2>&1 || exit $?
SGM_GROUP=4 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --frames 16 --no-cpu-baseline > gpurun_out/b_g4f16.log 2>&1 || exit $?
