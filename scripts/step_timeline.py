"""Critical path of the overlapped training step from a rocprofv3 kernel trace.

``python scripts/step_timeline.py <run_results.db> [sim_kernel_substring]``

In the overlapped bench step (``act_on_sim_stream``) the simulator stream runs act(t) -> explore(t) ->
simulator(t); the learner stream runs update(t) concurrently.  The wall step is therefore the gap between
two simulator kernel starts; this prints, per step inside the roctx ``bench_timed`` window (all steps when
the range is absent):

* ``sim``: the simulator kernel's duration,
* ``gap``: simulator end -> next simulator start (the act path, explore, handoff waits and launch gaps),
* the kernels on the simulator's stream inside that gap (the act path) with their durations,
* ``learn_end``: when the learner stream's last kernel of the step ended, relative to the simulator end
  (positive: the learner was the longer chain and the next act waited for it).
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "sim_step_kernel"
    c = sqlite3.connect(db)
    win = None
    try:
        win = c.execute("select start, end from regions where name like '%bench_timed%' or extdata like "
                        "'%bench_timed%' order by start limit 1").fetchone()
    except sqlite3.OperationalError:
        pass
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    if win:
        rows = [r for r in rows if r[2] >= win[0] and r[3] <= win[1]]
    sims = [r for r in rows if key in r[0]]
    if len(sims) < 2:
        print("fewer than two simulator kernels in the window")
        return
    sim_stream = sims[0][1]
    print(f"{len(sims)} simulator kernels on stream {sim_stream}; times in us")
    gaps, durs, learn = [], [], []
    agg = defaultdict(float)
    for a, b in zip(sims, sims[1:]):
        durs.append((a[3] - a[2]) / 1e3)
        gaps.append((b[2] - a[3]) / 1e3)
        inside = [r for r in rows if r[1] == sim_stream and r[2] >= a[3] and r[3] <= b[2]]
        for r in inside:
            agg[r[0][:90]] += (r[3] - r[2]) / 1e3
        other = [r for r in rows if r[1] != sim_stream and a[2] <= r[2] < b[2]]
        if other:
            learn.append((max(r[3] for r in other) - a[3]) / 1e3)
    n = len(gaps)
    print(f"sim {sum(durs) / n:8.1f}   gap (sim end -> next sim start) {sum(gaps) / n:7.1f}   "
          f"step {sum(durs) / n + sum(gaps) / n:8.1f}")
    if learn:
        print(f"learner stream's last kernel of the step ends {sum(learn) / len(learn):+.1f} us after the simulator")
    print("simulator-stream kernels inside the gap (us per step):")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"  {v / n:8.1f}  {k}")


if __name__ == "__main__":
    main()
