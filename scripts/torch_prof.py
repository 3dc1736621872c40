#!/usr/bin/env python
"""Attribute device time of the flagship training step to PyTorch ops (torch.profiler).

    python scripts/torch_prof.py [--envs 256] [--steps 5] [--no-overlap] [--rows 40]

Prints the ops with the largest self device time (with input shapes), complementing the
per-kernel rocprofv3 tables in profiles/.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=40)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--trace", default=None, help="write a chrome trace here")
    ap.add_argument("--by-count", action="store_true", help="sort framework ops by call count")
    a = ap.parse_args()
    import torch
    import yaml
    from torch.profiler import ProfilerActivity, profile

    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    os.chdir(ROOT)
    cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
    sim = load_batched_from_paths(["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                                  "configs/service_functions/abc.yaml", "configs/config/simulator/sample_config.yaml",
                                  cfg, a.envs, device="cuda")
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=a.envs, learning_starts=1, check_every=0,
                                                overlap_sim=not a.no_overlap, cuda_graphs=False))
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(a.steps):
            tr.step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60,
                   max_shapes_column_width=70))
    # framework ops with full input shapes, by self device time per step
    rows = [e for e in ka if e.key.startswith("aten::") and e.self_device_time_total > 0]
    rows.sort(key=lambda e: -e.count if a.by_count else -e.self_device_time_total)
    print(f"{'us/step':>9} {'calls/step':>10}  op  shapes")
    for e in rows[:a.rows]:
        print(f"{e.self_device_time_total / a.steps:9.1f} {e.count / a.steps:10.1f}  {e.key}  {e.input_shapes}")
    if a.trace:
        prof.export_chrome_trace(a.trace)


if __name__ == "__main__":
    main()
