#!/bin/bash
# variants.sh V1 V2 ... — C3 bench (pipelined + unpipelined) of the in-tree build ("base") and
# of lib/variants/lib_V.so for each V; one summary line per run in gpurun_out/variants.txt
set -u
mkdir -p gpurun_out
: > gpurun_out/variants.txt
run() {  # run NAME LIB ARGS
  local n=$1 lib=$2; shift 2
  SGM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/v_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/v_$n.log; exit 1; }
  python - "$n" "$*" gpurun_out/v_$n.log >> gpurun_out/variants.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
st = ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages'])
print(f"{sys.argv[1]:>14} {sys.argv[2]:>14} {d['value']:8.1f} pairs/s  {st}")
PY
}
for v in base "$@"; do
  lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so
  [ $v = base ] && lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
  run $v $lib
  run ${v}_np $lib --no-pipeline
done
cat gpurun_out/variants.txt
