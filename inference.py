#!/usr/bin/env python
"""Greedy inference with a trained actor (reference ``inference.py``: loads ``agent_helper.obj`` +
``trained_actor.pt`` from a hard-coded results dir and runs one episode on the inference network).

    python inference.py <run_dir> [--episodes 1] [--network <graphml>] [--envs 0] [--device cuda]

``--envs 0`` (default) steps one :class:`GymEnv` over the scalar simulator (test-mode CSVs are
written into ``<run_dir>/inference-<time>/``); ``--envs N`` runs N lockstep envs of the batched
device simulator with the greedy actor and reports the whole-batch success ratio.
Both files load without unpickling (JSON + ``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--episodes", type=int, default=1)
    ap.add_argument("--network", default=None, help="override the scheduler's inference network")
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--device", default=None)
    ap.add_argument("--seed", type=int, default=None)
    args = ap.parse_args(argv)

    import numpy as np
    import torch

    from gsc_amd.coordsim import reader
    from gsc_amd.models import GraphSet
    from gsc_amd.utils.checkpoint import load_actor, load_agent_helper

    dev = torch.device(args.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    h = load_agent_helper(os.path.join(args.run_dir, "agent_helper.obj"))
    actor, hdr = load_actor(os.path.join(args.run_dir, "trained_actor.pt"), dev)
    network = args.network or h.schedule["inference_network"]
    seed = h.seed if args.seed is None else args.seed
    sim_cfg = reader.get_config(h.sim_config_path)
    topo = reader.load_topology(network, sim_cfg)
    graphs = GraphSet([topo], hdr["n_pad"], dev)
    masks = graphs.action_masks(hdr["C"], hdr["F"])
    results = []
    if args.envs > 0:
        from gsc_amd.sim.batched import load_batched_from_paths
        sim = load_batched_from_paths([network], h.service_path, h.sim_config_path, h.config, args.envs, device=dev,
                                      seed=seed)
        obs = sim.reset().clone()
        topo_t = torch.zeros(args.envs, dtype=torch.int64, device=dev)
        succ = drop = 0.0
        t0 = time.perf_counter()
        with torch.no_grad():
            for _ in range(args.episodes * sim.episode_steps):
                a = actor(obs, topo_t, graphs, masks).float()
                out = sim.step(a)
                succ += float(out.stats[:, 0].sum())
                drop += float(out.stats[:, 1].sum())
                obs.copy_(out.obs)
        dt = time.perf_counter() - t0
        results.append({"envs": args.envs, "success_ratio": succ / max(succ + drop, 1.0),
                        "env_steps_per_s": args.envs * args.episodes * sim.episode_steps / dt})
    else:
        from gsc_amd.envs import GymEnv
        h.config_dir = os.path.join(args.run_dir, f"inference-{time.strftime('%Y-%m-%d_%H-%M-%S')}") + os.sep
        os.makedirs(h.config_dir, exist_ok=True)
        sched = dict(h.schedule, inference_network=network)
        env = GymEnv(h.config, sched, network, h.service_path, seed=seed, agent_helper=h,
                     sim_config_file=h.sim_config_path, test_mode=True)
        for ep in range(args.episodes):
            obs, _ = env.reset(seed=seed)
            ret, succ, drop = 0.0, 0, 0
            for _ in range(h.episode_steps):
                x = torch.zeros(1, hdr["n_pad"], hdr["obs_dim"], device=dev)
                x[0, :obs.num_nodes] = obs.x.to(dev)
                with torch.no_grad():
                    a = actor(x, torch.zeros(1, dtype=torch.int64, device=dev), graphs, masks)[0].float().cpu().numpy()
                obs, r, done, _, _ = env.step(np.asarray(a))
                st = env.current_simulator_state.network_stats
                succ += st["run_successful_flows"]
                drop += st["run_dropped_flows"]
                ret += float(r)
                if done:
                    break
            results.append({"episode": ep, "return": ret, "success_ratio": succ / max(succ + drop, 1)})
        env.close()
    for r in results:
        print(json.dumps(r))
    return results


if __name__ == "__main__":
    main()
