"""Env-steps/s of the batched simulator alone (fixed random schedule), for profiling."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
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
ap.add_argument("--profile", action="store_true")
ap.add_argument("--simcfg", default="configs/config/simulator/sample_config.yaml")
ap.add_argument("--cus", type=int, default=0, help="run on a stream CU-masked to this many CUs (0: all)")
ap.add_argument("--cu-per-xcd", type=int, default=0,
                help="with --cus: take the CUs as this many per 32-CU XCD block instead of contiguous bits")
ap.add_argument("--preset", default=None, help="bench.py preset (network / service / simulator / agent config)")
ap.add_argument("--episode-steps", type=int, default=None, help="override the agent config's episode length "
                "(default: the preset's, else the config's)")
args = ap.parse_args()
if args.preset:
    from bench import PRESETS
    pre = PRESETS[args.preset]
    nets, svc, args.simcfg, agent = pre["network"], pre["service"], pre["sim_config"], pre["agent_config"]
else:
    nets, svc, agent = [args.net], "configs/service_functions/abc.yaml", "configs/config/agent/sample_agent.yaml"
cfg = yaml.safe_load(open(agent))
ep = args.episode_steps or (pre.get("episode_steps") if args.preset else None)
if ep:
    cfg["episode_steps"] = int(ep)
sim = load_batched_from_paths(nets, svc, args.simcfg, cfg, args.envs, device=args.device)
n, P = sim.topologies[0].n, sim.n_pad
rng = np.random.default_rng(0)
a = np.zeros((P, sim.C, sim.F, P))
a[:n, :, :, :n] = rng.random((n, sim.C, sim.F, n))
a = threshold_normalize(a.reshape(-1), P, 0.1, 2).astype(np.float32)
A = torch.from_numpy(np.tile(a, (args.envs, 1))).to(args.device)
if args.cus:
    cus = list(range(args.cus))
    if args.cu_per_xcd:
        cus = [c for c in range(sim.native.cu_count()) if c % 32 < args.cu_per_xcd][: args.cus]
    stream = torch.cuda.ExternalStream(sim.native.create_cu_masked_stream(cus))
    torch.cuda.set_stream(stream)
sim.reset()
for _ in range(5):
    sim.step(A)
if args.device == "cuda":
    torch.cuda.synchronize()
if args.profile:
    sim.enable_profiling()
t = time.perf_counter()
S = D = 0.0
for _ in range(args.steps):
    out = sim.step(A)
if args.device == "cuda":
    torch.cuda.synchronize()
dt = time.perf_counter() - t
sim.check_flags()
print(f"cus={args.cus or 'all'}{'/xcd' + str(args.cu_per_xcd) if args.cu_per_xcd else ''} envs={args.envs} steps={args.steps} state_bytes={sim.state_bytes} "
      f"lds_mode={sim.ctx.lds_mode} lds_per_env={sim.ctx.lds_per_env} "
      f"env_steps_per_s={args.envs * args.steps / dt:.1f} ms_per_step={dt / args.steps * 1e3:.3f}")
if args.profile:
    pr = sim.prof.double().cpu()
    p = pr[: args.envs * 4].view(-1, 4).sum(0)
    ty = pr[args.envs * 4:].view(args.envs, 64, 2).sum(0)
    names = ["free", "writer", "mmpp", "trace", "arrival", "handle", "decide", "forward", "process", "request",
             "finish", "retlink"]
    phases = {60: "copy-in (state HBM->LDS)", 61: "copy-out (LDS->HBM)", 62: "prologue",
              57: "  of which topology stage + action load", 63: "epilogue"}
    tot = ty[:56, 0].sum()
    for i in range(56):
        if ty[i, 1] > 0:
            print(f"  {names[i // 4]:8s} state {i % 4} events/env-step={ty[i, 1] / (args.envs * args.steps):7.1f} "
                  f"cycles/dispatch={ty[i, 0] / ty[i, 1]:7.0f} share={ty[i, 0] / tot:.3f}")
    for i, nm in phases.items():
        if ty[i, 1] > 0:
            print(f"  {nm:26s} cycles/env-step={ty[i, 0] / ty[i, 1]:9.0f}")
    per = pr[args.envs * 4:].view(args.envs, 64, 2)
    t0s, t1s = per[:, 56, 0], per[:, 56, 1]
    if float(t1s.max()) > 0:  # the last step's wave start skew and durations (100 MHz ticks -> us)
        b = (t0s - t0s.min()) / 100.0
        d = (t1s - t0s) / 100.0
        q = torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.float64)
        print(f"  last step: wave start offset us (min/med/p90/max) {[round(float(x), 1) for x in b.quantile(q)]}  "
              f"wave duration us {[round(float(x), 1) for x in d.quantile(q)]}  "
              f"kernel span us {float((t1s.max() - t0s.min()) / 100.0):.1f}")
    if ty[59, 0] > 0:  # whole-workgroup shader cycles / 100 MHz wall ticks
        print(f"  effective engine clock  {ty[58, 0] / ty[59, 0] * 100:.0f} MHz")
    print(f"cycles/event: select={p[0] / p[3]:.0f} dispatch={p[1] / p[3]:.0f} merge={p[2] / p[3]:.0f} "
          f"events/env-step={p[3] / (args.envs * args.steps):.0f}  "
          f"event loop cycles/env-step={(p[0] + p[1] + p[2]) / (args.envs * args.steps):.0f}")
