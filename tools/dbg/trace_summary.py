import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
for name, us in seq:
    print(f"{us:10.1f} us  {name[:110]}")
