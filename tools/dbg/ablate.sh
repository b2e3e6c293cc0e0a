set -u
for v in ABL_BARRIER ABL_COSTDABL_STORE ABL_NOHORIZ; do
  SGM_HIP_LIB=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/ab_$v.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/ab_none.log 2>&1
