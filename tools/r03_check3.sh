mkdir -p gpurun_out; rm -f gpurun_out/ab_single.jsonl
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
bash tools/ab_single.sh c2,c3 2 diag80 diag96 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
