"""Summarise a rocprofv3 kernel-trace database: per-kernel total/mean time per timed step.

``python scripts/prof_summary.py <run_results.db> <steps> [top]``.  When the database holds the
``bench_timed`` roctx range (``GSC_PROF_WINDOW=1 rocprofv3 --kernel-trace --marker-trace ...
bench.py``) only kernels that start and end inside it are counted, so init work and warm-up steps
are excluded and the per-step numbers are exact; otherwise the whole process is divided by
``steps`` (and the header says so).
"""
import glob
import sqlite3
import sys

db = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/prof/*.db")[0]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
c = sqlite3.connect(db)
win = None
try:
    win = c.execute("select start, end from regions where extdata like '%bench_timed%' or name like '%bench_timed%' order by start limit 1").fetchone()
except sqlite3.OperationalError:
    pass
where, args = "", ()
if win:
    where, args = "where start >= ? and end <= ?", tuple(win)
rows = c.execute(f"select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels {where} group by name "
                 "order by sum(end-start) desc", args).fetchall()
tot = sum(r[2] for r in rows)
if win:
    wall = (win[1] - win[0]) / 1e3
    print(f"timed region only (roctx bench_timed): wall {wall / steps:.1f} us/step, "
          f"kernel time {tot / steps:.1f} us/step (sum over streams) over {steps:.0f} steps")
else:
    print(f"WHOLE PROCESS (no bench_timed range): total kernel time {tot / 1e3:.2f} ms / {steps:.0f} steps "
          f"= {tot / steps / 1e3:.3f} ms/step (includes init + warm-up)")
print(f"{'us/step':>9} {'calls/step':>10} {'us/call':>9}  kernel")
for r in rows[:top]:
    print(f"{r[2] / steps:9.1f} {r[1] / steps:10.1f} {r[3]:9.1f}  {r[0][:100]}")
