#!/bin/bash
# env_variants.sh "ENV=.. ENV2=.." ... — C3 bench of the in-tree build under each environment,
# interleaved over ROUNDS (default 2) rounds; one line per run in gpurun_out/env_variants.txt
set -u
mkdir -p gpurun_out
: > gpurun_out/env_variants.txt
i=0
for rnd in $(seq ${ROUNDS:-2}); do
for e in "" "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/e_$i.log 2>&1 || { echo "[$e] failed"; tail -5 gpurun_out/e_$i.log; exit 1; }
  python - "$e" gpurun_out/e_$i.log >> gpurun_out/env_variants.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
st = ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages'])
print(f"[{sys.argv[1]:>24}] {d['value']:8.1f} pairs/s  {st}")
PY
done
done
sort -s -k1,1 gpurun_out/env_variants.txt
