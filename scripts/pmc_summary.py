"""Summarise a rocprofv3 --pmc CSV (counter_collection.csv): per-kernel mean of each counter per dispatch."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
dur = {}
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
    dur[(k, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = defaultdict(float)
for (k, _), d in dur.items():
    tot[k] += d
names = sorted(tot, key=lambda k: -tot[k])[:top]
ctrs = sorted({c for k in names for c in acc[k]})
for k in names:
    n = len(disp[k])
    print(f"{k[:100]}\n  dispatches={n} mean_us={tot[k] / n / 1e3:.1f}")
    for c in ctrs:
        print(f"    {c:24s} {acc[k][c] / n:16.1f}")
