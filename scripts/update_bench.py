#!/usr/bin/env python
"""Learner-only timing of the graphed native DDPG update at a bench preset's shapes (no simulator).

Random batch of the preset's size (B = 100 x 256 envs), ``--iters`` replays of the captured update timed with
HIP events; ``GSC_UPDATE_BRANCHES`` selects the concurrent-branch update (default) or one serial chain.

    python scripts/update_bench.py --preset abilene --iters 50
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PRESETS = {
    "abilene": (["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"], "configs/config/agent/sample_agent.yaml",
                "configs/service_functions/abc.yaml"),
    "syn50": (["configs/networks/synthetic/syn50-in8-cap1-3.graphml"], "configs/config/agent/agent_syn50.yaml",
              "configs/service_functions/abc-3sfc.yaml"),
    "syn200": ([f"configs/networks/synthetic/syn200-in16-cap1-3-s{i}.graphml" for i in range(3)],
               "configs/config/agent/agent_syn200.yaml", "configs/service_functions/abc-3sfc.yaml"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(PRESETS), default="abilene")
    ap.add_argument("--batch", type=int, default=25600)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch
    import yaml
    from gsc_amd.agents import Batch, DDPGLearner
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GraphSet
    from gsc_amd.sim.batched import load_batched_from_paths
    os.chdir(ROOT)
    nets, agent, svc = PRESETS[a.preset]
    cfg = yaml.safe_load(open(agent))
    sim = load_batched_from_paths(nets, svc, "configs/config/simulator/sample_config.yaml", cfg, 1, device="cuda")
    gs = GraphSet([load_topology(p) for p in nets], sim.n_pad, "cuda")
    L = DDPGLearner(cfg, sim.n_obs, sim.action_dim, gs, sim.C, sim.F, "cuda", seed=1)
    B, P, A = a.batch, sim.n_pad, sim.action_dim
    g = torch.Generator(device="cuda").manual_seed(0)
    topo = torch.randint(0, gs.num_topologies, (B,), device="cuda", generator=g)
    obs = torch.rand(B, P, sim.n_obs, device="cuda", generator=g) * gs.node_mask[topo].unsqueeze(-1)
    nxt = torch.rand(B, P, sim.n_obs, device="cuda", generator=g) * gs.node_mask[topo].unsqueeze(-1)
    acts = torch.rand(B, (A + 7) // 8 * 8, device="cuda", generator=g).to(torch.bfloat16)
    b = Batch(obs, topo, acts, torch.rand(B, device="cuda", generator=g), nxt, torch.zeros(B, device="cuda"))
    for _ in range(4):   # eager warm-up, then capture
        L.update_graphed(b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        L.update_graphed(b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"{a.preset} B={B} branches={os.environ.get('GSC_UPDATE_BRANCHES', '1')} update {ms * 1e3:.1f} us "
          f"finite={bool(torch.isfinite(L.critic_flat.flat).all())}", flush=True)


if __name__ == "__main__":
    main()
