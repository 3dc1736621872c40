#!/usr/bin/env python
"""Per-step timeline from a rocprofv3 kernel-trace database.

    python scripts/timeline.py gpurun_out/prof/run_results.db [--steps 5]

Steps are delimited by the simulator kernel; for each of the last N steps prints the simulator
kernel interval, the busy time / span of all other kernels, and idle gaps on the device.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    sims = [r for r in rows if "sim_step_kernel" in r[0]]
    if len(sims) < 2:
        print("no simulator kernels found; columns:", cols)
        return
    for k in range(max(0, len(sims) - a.steps - 1), len(sims) - 1):
        t0, t1 = sims[k][1], sims[k + 1][1]
        ks = [r for r in rows if t0 <= r[1] < t1]
        sim = sims[k]
        other = [r for r in ks if "sim_step_kernel" not in r[0]]
        # union of intervals of non-sim kernels
        iv = sorted((r[1], r[2]) for r in other)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        before = [r for r in other if r[2] <= sim[1]]
        print(f"step {k}: period {(t1 - t0) / 1e3:8.1f} us | sim {(sim[2] - sim[1]) / 1e3:7.1f} us "
              f"(starts +{(sim[1] - t0) / 1e3:.1f}) | other kernels {len(other):4d} busy {busy / 1e3:7.1f} us "
              f"| {len(before)} kernels end before the sim starts")
        if k == len(sims) - 2:
            print("  first 12 non-sim kernels of the last step (offset us, dur us):")
            for r in other[:12]:
                print(f"    +{(r[1] - t0) / 1e3:8.1f} {(r[2] - r[1]) / 1e3:7.1f}  {r[0][:70]}")
            print("  gaps > 20 us between consecutive non-sim kernels:")
            last_end = None
            for r in other:
                if last_end is not None and r[1] - last_end > 20e3:
                    print(f"    gap {(r[1] - last_end) / 1e3:7.1f} us before +{(r[1] - t0) / 1e3:.1f} {r[0][:60]}")
                last_end = max(last_end or 0, r[2])


if __name__ == "__main__":
    main()
