# full GPU suite, then the shipped-config OCV timings
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 400 python -u tools/ocv_modes_bench.py --reps 10 --case "${CASE:-refcfg}" > gpurun_out/ocv_ref.jsonl 2> gpurun_out/ocv_ref.err || { tail -20 gpurun_out/ocv_ref.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/ocv_ref.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["case"][:70], d["gpu_ms_per_frame"], [(s["name"], s["avg_ms"]) for s in d["stages"]])
PY
