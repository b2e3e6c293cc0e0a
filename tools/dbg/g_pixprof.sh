# kernel trace + a VALU/LDS PMC pass of the OCV cost stage on the shipped config
set -u
export TMPDIR=/tmp
O=gpurun_out/pixprof; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/ocv_modes_bench.py --reps 3 --case "MODE_SGBM (gated)" > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/stats.csv
cut -d, -f1-4 $O/stats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/pmc -o run --output-format csv -- python3 tools/ocv_modes_bench.py --reps 2 --case "MODE_SGBM (gated)" > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pixprof/pmc/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:40]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in acc.items():
    c = n[(k, 'SQ_WAVES')] or 1
    print(k, {m: round(v / c / 1e6, 2) for m, v in d.items()})
PY
