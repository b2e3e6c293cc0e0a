"""Timeline of a rocprofv3 kernel + memory-copy trace: per kernel its duration and the idle
gap before it, and the copies overlapping; summary of GPU busy vs idle."""
import csv
import glob
import sys

d = sys.argv[1]
kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
mf = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(kf[0]))))
ms = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "?"))) for r in csv.DictReader(open(mf[0])))) if mf else []
big = [k for k in ks if (k[1] - k[0]) > 200_000]   # > 0.2 ms: the pipeline launches
print("kernels", len(ks), "big", len(big), "copies", len(ms))
if ms:
    import collections
    c = collections.defaultdict(list)
    for a, b, n in ms:
        c[n].append((b - a) / 1e3)
    for n, v in c.items():
        print("copy", n, len(v), "avg us %.1f max %.1f" % (sum(v) / len(v), max(v)))
# take the last 70 big kernels (steady state of the last step)
tail = ks[-400:]
prev_end = None
busy = idle = 0
for a, b, n in tail:
    if prev_end is not None:
        gap = a - prev_end
        if gap > 0:
            idle += gap
        if gap > 50_000:
            print(f"gap {gap/1e3:8.1f} us before {n}")
    busy += b - a
    prev_end = max(prev_end or 0, b)
print(f"tail: busy {busy/1e6:.2f} ms idle {idle/1e6:.2f} ms")
for a, b, n in tail[-40:]:
    print(f"{(b-a)/1e3:9.1f} us {n}")
