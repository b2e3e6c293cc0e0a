set -u
mkdir -p gpurun_out
: > gpurun_out/ocv_var.txt
# VARIANTS: name[:ENV=VAL] ...; lib_<name>.so when it exists, else the in-tree build
for rnd in 1 2; do
for spec in ${VARIANTS:-base}; do
  v=${spec%%:*}; env=""; [ "$spec" != "$v" ] && env=${spec#*:}
  lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so
  [ -f $lib ] || lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
  env $env SGM_HIP_LIB=$lib timeout -k 10 300 python tools/ocv_modes_bench.py --reps 10 --case "${CASE-1920x1080}" > gpurun_out/ocv_$v.log 2>&1 || { tail -5 gpurun_out/ocv_$v.log; exit 1; }
  python3 - "$spec" $v >> gpurun_out/ocv_var.txt <<'P'
import json,sys
for l in open(f"gpurun_out/ocv_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d=json.loads(l); print(f"{sys.argv[1]:18s} {d['case'][:46]:46s} {d['gpu_ms_per_frame']:8.3f} ", ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages']))
P
done; done
sort -s -k1,1 gpurun_out/ocv_var.txt
