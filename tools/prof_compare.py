"""Per-launch-kind kernel durations from a rocprofv3 --kernel-trace CSV beside the HIP-event
stage averages bench.py printed in the same run (the agreement check of the roofline's
avg_launch_ms).

    python tools/prof_compare.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/rocprof.log
"""
import collections
import csv
import json
import sys


def main():
    trace, log = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(trace)))
    by = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = f"{name} grid={r['Grid_Size_X']}" if "fused" in name else name
        by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print("rocprofv3 kernel trace (ms per dispatch):")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:70s} n={len(v):4d} avg={sum(v) / len(v):8.4f} total={sum(v):9.3f}")
    bench = None
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            bench = json.loads(line)
    if bench:
        print("bench.py HIP events, same process (ms per launch):")
        for s in bench["stages"]:
            print(f"  {s['name']:70s} n={s['launches']:4d} avg={s['avg_ms']:8.4f}")
        print(f"bench value {bench['value']} pairs/s, roofline {json.dumps(bench['roofline'])}")


if __name__ == "__main__":
    main()
