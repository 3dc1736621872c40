"""Print the kernel dispatch sequence (name, grid, duration) of the last N dispatches of a rocprofv3
database -- maps each launch of a generic kernel (e.g. the MFMA GEMM) to its place in the update."""
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
skip_sim = "--all" not in sys.argv
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, start, end, stream_id from kernels "
                 "order by start").fetchall()
rows = rows[-n:]
t0 = rows[0][5]
for name, gx, gy, gz, wx, s, e, st in rows:
    if skip_sim and "sim_step" in name:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}us  [stream {st}] SIM")
        continue
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}us  [stream {st}] grid=({gx // wx},{gy},{gz}) {name[:80]}")
