set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_single.jsonl gpurun_out/ab_bench.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab_single.sh c2,c3,c5 2 edge0 || exit 1
for r in 1 2; do
  for v in base edge0; do
    if [ $v = base ]; then lib=""; else lib=i3dr_stereo_camera-ros_amd/lib/variants/$v/libsgm_hip.so; fi
    SGM_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep '^{' | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ab_bench.jsonl || exit 1
  done
done
