"""Env-steps/s of the batched simulator alone (fixed random schedule), for profiling."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import numpy as np
import torch
import yaml

from gsc_amd.envs import threshold_normalize
from gsc_amd.sim.batched import load_batched_from_paths

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=256)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--device", default="cuda")
ap.add_argument("--net", default="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml")
ap.add_argument("--simcfg", default="configs/config/simulator/sample_config.yaml")
args = ap.parse_args()
cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
sim = load_batched_from_paths([args.net], "configs/service_functions/abc.yaml", args.simcfg, cfg, args.envs,
                              device=args.device)
n = sim.topologies[0].n
rng = np.random.default_rng(0)
a = np.zeros((24, 1, 3, 24))
a[:n, :, :, :n] = rng.random((n, 1, 3, n))
a = threshold_normalize(a.reshape(-1), 24, 0.1, 2).astype(np.float32)
A = torch.from_numpy(np.tile(a, (args.envs, 1))).to(args.device)
sim.reset()
for _ in range(5):
    sim.step(A)
if args.device == "cuda":
    torch.cuda.synchronize()
t = time.perf_counter()
S = D = 0.0
for _ in range(args.steps):
    out = sim.step(A)
if args.device == "cuda":
    torch.cuda.synchronize()
dt = time.perf_counter() - t
sim.check_flags()
print(f"envs={args.envs} steps={args.steps} state_bytes={sim.state_bytes} lds={sim.ctx.use_lds} "
      f"env_steps_per_s={args.envs * args.steps / dt:.1f} ms_per_step={dt / args.steps * 1e3:.3f}")
