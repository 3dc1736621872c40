"""Per-kernel duration table of a rocprofv3 database: python scripts/diag/kstats.py <run_results.db> [n]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for r in c.execute("select name, count(*), avg(duration)/1000.0, min(duration)/1000.0 from kernels group by name "
                   "order by sum(duration) desc limit ?", (n,)):
    print(f"{r[0][:80]:80s} n={r[1]:5d} avg {r[2]:9.1f} us  min {r[3]:9.1f} us")
