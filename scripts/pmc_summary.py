"""Mean PMC counter value per dispatch, per kernel, from rocprofv3 --pmc csv output(s)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"][:70]
        c = row["Counter_Name"]
        acc[k][c] += float(row["Counter_Value"])
        cnt[k][c].add(row["Dispatch_Id"])
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        print(f"    {c:32s} {acc[k][c] / max(1, len(cnt[k][c])):16.4g}")
