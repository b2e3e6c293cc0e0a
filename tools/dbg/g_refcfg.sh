set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_refcfg.py tests/test_gpu_ocv.py tests/test_gpu_fuzz.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ref.log 2>&1 || { tail -40 gpurun_out/t_ref.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_ref.log | tail -3
timeout -k 10 600 python tools/ocv_modes_bench.py --reps 5 > gpurun_out/ocv_modes.log 2>&1 || { tail -20 gpurun_out/ocv_modes.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/ocv_modes.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['case'], d['gpu_ms_per_frame'], [(s['name'], s['avg_ms'], s['frac']) for s in d['stages']])
"
