#!/usr/bin/env python
"""Experiment: simulator and learner on disjoint CU sets (CU-masked HIP streams).

For K CUs given to the simulator (the rest to the learner) measures: simulator step alone,
learner update alone, and both concurrently — per step, ms.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import yaml
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.native import load
    from gsc_amd.sim.batched import load_batched_from_paths
    nat = load()
    os.chdir(ROOT)
    E = int(os.environ.get("ENVS", "256"))
    cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
    sim = load_batched_from_paths(["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                                  "configs/service_functions/abc.yaml", "configs/config/simulator/sample_config.yaml",
                                  cfg, E, device="cuda")
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=E, learning_starts=1, check_every=0, overlap_sim=False))
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    act = tr.act_buf.clone()
    n = nat.cu_count()
    N = 10
    batch = tr.replay.sample(tr.batch_size)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e3

    base_sim = timed(lambda: sim.step(act))
    base_learn = timed(lambda: tr.learner.update(batch))
    print(f"all {n} CUs: sim {base_sim:.3f} ms  learner {base_learn:.3f} ms  serial sum {base_sim + base_learn:.3f}")
    for layout in ("contiguous", "interleaved"):
        for K in (32, 48, 64, 86, 96, 128):
            if layout == "contiguous":
                sim_cus = list(range(K))
            else:
                step = n / K
                sim_cus = sorted({int(i * step) for i in range(K)})
            rest = [c for c in range(n) if c not in set(sim_cus)]
            s_sim = torch.cuda.ExternalStream(nat.create_cu_masked_stream(sim_cus))
            s_learn = torch.cuda.ExternalStream(nat.create_cu_masked_stream(rest))

            def sim_only():
                with torch.cuda.stream(s_sim):
                    sim.step(act)

            def learn_only():
                with torch.cuda.stream(s_learn):
                    tr.learner.update(batch)

            def both():
                with torch.cuda.stream(s_sim):
                    sim.step(act)
                with torch.cuda.stream(s_learn):
                    tr.learner.update(batch)

            ts, tl, tb = timed(sim_only), timed(learn_only), timed(both)
            print(f"{layout:>11} K={K:3d}: sim {ts:.3f}  learner {tl:.3f}  concurrent {tb:.3f} ms", flush=True)
    # unpartitioned concurrency (two ordinary streams)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both_plain():
        with torch.cuda.stream(s1):
            sim.step(act)
        with torch.cuda.stream(s2):
            tr.learner.update(batch)
    print(f"unmasked streams concurrent {timed(both_plain):.3f} ms")


if __name__ == "__main__":
    main()
