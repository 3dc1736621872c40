"""Per-kernel mean counters of a rocprofv3 --pmc csv, plus VALU wave-instructions per CU-cycle
(SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x CUs)): ``python scripts/diag/pmc_table.py <csv> [filter] [cus]``"""
import collections
import csv
import sys

path, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
acc = collections.defaultdict(lambda: collections.defaultdict(float))
ids = collections.defaultdict(lambda: collections.defaultdict(set))
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    if filt not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    ids[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k, c in acc.items():
    m = {n: v / max(1, len(ids[k][n])) for n, v in c.items()}
    wall = m.get("GRBM_GUI_ACTIVE", 0) / 8
    extra = f" valu/CU-cycle={m['SQ_INSTS_VALU'] / (wall * cus):.2f}" if wall and "SQ_INSTS_VALU" in m else ""
    print(k, " ".join(f"{n}={v:.3g}" for n, v in sorted(m.items())) + extra)
