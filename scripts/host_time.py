#!/usr/bin/env python
"""Host-side cost of one training step: time spent in trainer.step() calls (no device sync) vs the
device period.  If host time per step >= period, the loop is launch-bound."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import yaml

from gsc_amd.agents import BatchedTrainer, TrainerConfig
from gsc_amd.sim.batched import load_batched_from_paths

os.chdir(ROOT)
cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
sim = load_batched_from_paths(["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                              "configs/service_functions/abc.yaml", "configs/config/simulator/sample_config.yaml",
                              cfg, 256, device="cuda")
tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=256, learning_starts=1, check_every=0))
for _ in range(10):
    tr.step()
torch.cuda.synchronize()
N = 40
host = []
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter()
    tr.step()
    host.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
host.sort()
print(f"host per step: median {host[N // 2] * 1e3:.3f} ms  min {host[0] * 1e3:.3f}  max {host[-1] * 1e3:.3f}; "
      f"enqueue loop {(t1 - t0) / N * 1e3:.3f} ms/step; wall {(t2 - t0) / N * 1e3:.3f} ms/step")
