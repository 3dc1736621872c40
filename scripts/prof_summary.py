"""Summarise a rocprofv3 kernel-trace database: per-kernel total/mean time (per timed step)."""
import glob
import sqlite3
import sys

db = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/prof/*.db")[0]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels group by name "
                 "order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot / 1e3:.2f} ms over {steps:.0f} steps = {tot / steps / 1e3:.3f} ms/step")
print(f"{'us/step':>9} {'calls/step':>10} {'us/call':>9}  kernel")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{r[2] / steps:9.1f} {r[1] / steps:10.1f} {r[3]:9.1f}  {r[0][:90]}")
