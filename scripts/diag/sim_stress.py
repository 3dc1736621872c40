#!/usr/bin/env python
"""Stress the batched simulator with concentrated (learned-like) schedules on the host path: every step draws
peaked random weights (u ** power), post-processes them with a given threshold (the opt-in schedule_threshold) and
checks the overflow / bad-state flags.  Diagnoses simulator faults that only non-uniform schedules reach (at 50-200
nodes the reference threshold makes every row uniform).

    python scripts/diag/sim_stress.py --preset syn50 --envs 8 --steps 400 --threshold 0.048 --power 6
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.chdir(ROOT)

import numpy as np
import torch
import yaml

from bench import PRESETS
from gsc_amd.ops import explore_postprocess
from gsc_amd.models.graphs import GraphSet
from gsc_amd.sim.batched import load_batched_from_paths

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="syn50")
ap.add_argument("--envs", type=int, default=8)
ap.add_argument("--steps", type=int, default=400)
ap.add_argument("--threshold", type=float, default=0.048)
ap.add_argument("--power", type=float, default=6.0)
ap.add_argument("--device", default="cpu")
ap.add_argument("--seed", type=int, default=0)
a = ap.parse_args()
pre = PRESETS[a.preset]
cfg = yaml.safe_load(open(pre["agent_config"]))
if pre.get("episode_steps"):
    cfg["episode_steps"] = pre["episode_steps"]
sim = load_batched_from_paths(pre["network"], pre["service"], pre["sim_config"], cfg, a.envs, device=a.device,
                              seed=a.seed)
graphs = GraphSet(sim.topologies, sim.n_pad, sim.device)
masks = graphs.action_masks(sim.C, sim.F)
g = torch.Generator(device=a.device).manual_seed(a.seed)
sim.reset()
topo = torch.zeros(a.envs, dtype=torch.int64, device=a.device)
t0 = time.time()
for step in range(a.steps):
    mu = torch.rand(a.envs, sim.action_dim, device=a.device, generator=g) ** a.power
    act = explore_postprocess(mu * masks[topo], masks, sim.n_pad, False, 0.0, 0.0, seed=a.seed, step=step,
                              topo=topo, threshold=a.threshold)
    out = sim.step(act, buffer_set=step & 1)
    if (step + 1) % sim.episode_steps == 0:
        topo = sim.topo_next.to(torch.int64).clone()
    sim.check_flags()
    if step % 50 == 0:
        print(f"step {step} ok ({time.time() - t0:.1f} s)", flush=True)
print(f"done: {a.steps} steps, {a.envs} envs, threshold {a.threshold}, power {a.power}")
