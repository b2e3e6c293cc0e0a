"""Kernel durations and the idle gaps between consecutive dispatches of a rocprofv3
--kernel-trace CSV (one stream), averaged per kernel name over the last --tail dispatches:
how much of a single frame's wall time is kernels and how much launch gaps.

    python tools/trace_gaps.py gpurun_out/sf/run_kernel_trace.csv [--tail 60]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=60)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.tail:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[name].append((e - s) / 1e3)
        if prev_end is not None:
            gap[name].append((s - prev_end) / 1e3)
        prev_end = e
    print(f"{'kernel':60s} {'n':>4s} {'avg us':>9s} {'gap before us':>14s}")
    for k, v in dur.items():
        g = gap.get(k, [0.0])
        print(f"{k:60s} {len(v):4d} {sum(v) / len(v):9.2f} {sum(g) / len(g):14.2f}")


if __name__ == "__main__":
    main()
