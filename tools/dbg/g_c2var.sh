set -u
mkdir -p gpurun_out
: > gpurun_out/c2var.txt
for rnd in 1 2; do
for v in base lpl8; do
  lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so
  [ $v = base ] && lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
  for cfg in c2 c3; do
    SGM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg > gpurun_out/v_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/v_$v.log; exit 1; }
    python3 - "$v $cfg" gpurun_out/v_$v.log >> gpurun_out/c2var.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
st = ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages'])
print(f"{sys.argv[1]:>12} {d['value']:8.1f} pairs/s  {st}")
PY
  done
done; done
sort -s -k1,2 gpurun_out/c2var.txt
