# fused-launch WTA interleave period sweep (C3 bench, pipelined)
set -u
for P in ${PERIODS:-0 2 3 4 6 10}; do
  SGM_WTA_PERIOD=$P timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p$P.log 2>&1 || exit $?
  echo "P=$P $(tail -1 gpurun_out/p$P.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], [(s["name"], s["avg_ms"]) for s in d["stages"]])')"
done
