set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
for v in 1 0; do
  SGM_UPWTA=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_up$v.log 2>&1 || { tail -20 gpurun_out/b_up$v.log; exit 1; }
done
for v in 1 0; do
  SGM_UPWTA=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --config c2 > gpurun_out/b_c2_up$v.log 2>&1 || { tail -20 gpurun_out/b_c2_up$v.log; exit 1; }
done
python - <<'P'
import json
for f in ("b_up1","b_up0","b_c2_up1","b_c2_up0"):
    l=[x for x in open("gpurun_out/"+f+".log") if x.startswith("{")][-1]; d=json.loads(l)
    print(f, d["value"], d["ms_per_frame"], (d["roofline"] or {}).get("frac"), ' '.join(f"{s['name']}={s['avg_ms']:.3f}" for s in d['stages']))
P
