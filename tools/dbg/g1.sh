set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_census.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_batch.log 2>&1 || { tail -40 gpurun_out/t_batch.log; exit 1; }
tail -5 gpurun_out/t_batch.log
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_dev.log 2>&1 || { tail -20 gpurun_out/b_dev.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --host-io > gpurun_out/b_host.log 2>&1 || { tail -20 gpurun_out/b_host.log; exit 1; }
python - <<'P'
import json
for f in ("gpurun_out/b_dev.log","gpurun_out/b_host.log"):
    l=[x for x in open(f) if x.startswith("{")][-1]; d=json.loads(l)
    print(f, d["value"], d["ms_per_frame"], (d["roofline"] or {}).get("frac"))
P
