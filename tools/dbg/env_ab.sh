# env_ab.sh "ENV1" "ENV2" ... — C3 bench under each environment, interleaved over ROUNDS rounds
set -u
mkdir -p gpurun_out
: > gpurun_out/env_ab.txt
for rnd in $(seq ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/env_$i.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/env_$i.log; exit 1; }
    python3 - "$e" gpurun_out/env_$i.log >> gpurun_out/env_ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
st = ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages'])
print(f"{sys.argv[1]:>24} {d['value']:8.1f} pairs/s frac {d['roofline']['frac']:.4f}  {st}")
PY
  done
done
sort -s -k1,1 gpurun_out/env_ab.txt
