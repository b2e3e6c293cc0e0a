#!/bin/bash
# variants.sh [-n] V1 V2 ... — C3 bench of the in-tree build ("base") and of
# lib/variants/lib_V.so for each V, interleaved over ROUNDS (default 3) rounds so clock and
# thermal drift hits every variant alike; -n adds the unpipelined (--no-pipeline) runs.
# One summary line per run in gpurun_out/variants.txt.
set -u
mkdir -p gpurun_out
: > gpurun_out/variants.txt
NP=0
if [ "${1:-}" = -n ]; then NP=1; shift; fi
run() {  # run NAME LIB ARGS
  local n=$1 lib=$2; shift 2
  SGM_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/v_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/v_$n.log; exit 1; }
  python - "$n" "$*" gpurun_out/v_$n.log >> gpurun_out/variants.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
st = ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages'])
print(f"{sys.argv[1]:>14} {sys.argv[2]:>14} {d['value']:8.1f} pairs/s  {st}")
PY
}
for rnd in $(seq ${ROUNDS:-3}); do
  for v in base "$@"; do
    lib=i3dr_stereo_camera-ros_amd/lib/variants/lib_$v.so
    [ $v = base ] && lib=i3dr_stereo_camera-ros_amd/lib/libsgm_hip.so
    run $v $lib
    [ $NP = 1 ] && run ${v}_np $lib --no-pipeline
  done
done
sort -s -k1,1 gpurun_out/variants.txt
