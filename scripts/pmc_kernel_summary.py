#!/usr/bin/env python
"""Per-kernel mean of every counter in a rocprofv3 --pmc counter_collection.csv, with per-wave ratios.

    python scripts/pmc_kernel_summary.py gpurun_out/ex/pmc/run_counter_collection.csv explore
"""
import collections
import csv
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(disp[k])
        mean = {c: x / n for c, x in v.items()}
        waves = mean.get("SQ_WAVES", 0)
        print(f"{k[:90]}  dispatches {n}")
        for c in sorted(mean):
            per = f"  per wave {mean[c] / waves:.1f}" if waves and c != "SQ_WAVES" else ""
            print(f"  {c:24s} {mean[c]:.4g}{per}")


if __name__ == "__main__":
    main()
