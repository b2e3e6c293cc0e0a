set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_refcfg.py tests/test_gpu_ocv.py tests/test_gpu_fuzz.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ocv.log 2>&1 || { tail -40 gpurun_out/t_ocv.log; exit 1; }
tail -2 gpurun_out/t_ocv.log
rm -rf gpurun_out/prof_ref
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o run --output-format csv -- python3 tools/ocv_modes_bench.py --reps 5 --case "gated" > gpurun_out/ocv_ref.log 2>&1 || { tail gpurun_out/ocv_ref.log; exit 1; }
grep '^{' gpurun_out/ocv_ref.log | cut -c1-300
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/prof_ref/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)): print(r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us', r['Percentage'])
"
rm -rf gpurun_out/prof_ref
