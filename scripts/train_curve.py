#!/usr/bin/env python
"""Short batched training run; prints success ratio / losses per lockstep episode (learning check).

``--fp32`` runs the fp32 autograd learner (no bf16 operands; with GSC_GNN_NATIVE=0 the embedder is
the PyTorch reference too); GSC_COMPOSE=0 selects the materialised critic(obs, actor(obs)) actor
loss; ``--ref-ratio`` performs E updates of batch 100 per lockstep step (the reference's update
rule: one batch-100 update per env step) instead of one update of batch 100 * E."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=20)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--agent", default="configs/config/agent/sample_agent.yaml")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--ref-ratio", action="store_true")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    import yaml
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    os.chdir(ROOT)
    cfg = yaml.safe_load(open(a.agent))
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    sim = load_batched_from_paths(["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                                  "configs/service_functions/abc.yaml", "configs/config/simulator/sample_config.yaml",
                                  cfg, a.envs, device=dev, seed=a.seed)
    kw = dict(batch_size=100, updates_per_step=a.envs) if a.ref_ratio else {}
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=a.envs, seed=a.seed, check_every=0,
                                                amp_bf16=False if a.fp32 else None, **kw))
    for ep in range(a.episodes):
        for _ in range(sim.episode_steps):
            tr.step()
        m = tr.metrics()
        print(f"{a.tag} ep {ep:3d} success {m['success_ratio']:.4f} return {m['mean_episode_return']:8.2f} "
              f"qf1 {m.get('qf1_loss', float('nan')):.4f} actor {m.get('actor_loss', float('nan')):.4g} "
              f"q {m.get('qf1_values', float('nan')):.4g}", flush=True)


if __name__ == "__main__":
    main()
