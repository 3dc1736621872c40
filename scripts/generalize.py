#!/usr/bin/env python
"""Generalisation check for the large-topology configs (BASELINE configs 4 / 5): train on scheduler-switched
topologies, test on a held-out one against random and uniform schedules.

The reference trains with the network scheduler swapping the training network between episodes
(``/root/reference/src/rlsp/envs/gym_env.py:103-128``) and tests the trained actor on an unseen
``inference_network`` (``/root/reference/main.py:61-76``).  Here:

* train: ``BatchedTrainer`` on the preset's training topologies, every env switched to the next topology every
  ``period`` episodes (1 for syn50 / syn200, the reference's 10 for its scheduler_type presets), bounded actor (``actor_output_activation: sigmoid``,
  docs/DEVIATIONS.md Q6), ``--train-steps`` lockstep steps of ``--envs`` envs;
* test: ``--eval-envs`` envs on the held-out topology, one episode each (``--eval-envs`` episodes), for three
  schedules post-processed exactly like the reference's actions (simple_ddpg.py:374-395):
  ``trained`` = the greedy actor (no exploration noise), ``random`` = uniform random weights per destination
  (the warm-up policy), ``uniform`` = equal weights on every real destination;
  success ratio = successful / (successful + dropped) flows over all test episodes.

Prints one JSON line per seed.

    python scripts/generalize.py --preset syn50 --seed 0 --train-steps 8000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NET = "configs/networks/synthetic"
PRESETS = {
    # 50-node: three training variants, the fourth held out; Poisson arrivals at the ingress nodes
    "syn50": dict(train=[f"{NET}/syn50-in8-cap1-3.graphml", f"{NET}/syn50-in8-cap1-3-s1.graphml",
                         f"{NET}/syn50-in8-cap1-3-s2.graphml"],
                  test=f"{NET}/syn50-in8-cap1-3-s3.graphml", agent="configs/config/agent/agent_syn50.yaml",
                  service="configs/service_functions/abc-3sfc.yaml",
                  sim="configs/config/simulator/sample_config.yaml", episode_steps=50),
    # the reference's own generalisation schedulers (configs/config/scheduler_type{1,2,4}.yaml): their training
    # networks (period 10 episodes) and inference network, Abilene-scale (n_pad 24), abc service, 200-step episodes
    "type1": dict(train=["configs/networks/abilene/abilene-in4-rand-cap0-2.graphml",
                         "configs/networks/abilene/abilene-in4-cap1.graphml"],
                  test="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml",
                  agent="configs/config/agent/sample_agent.yaml", service="configs/service_functions/abc.yaml",
                  sim="configs/config/simulator/sample_config.yaml", episode_steps=200, period=10),
    "type2": dict(train=["configs/networks/abilene/abilene-in4-rand-cap.graphml",
                         "configs/networks/abilene/abilene-in4-rand-cap0-2.graphml"],
                  test="configs/networks/abilene/abilene-in4-rand-cap1-2-perm1.graphml",
                  agent="configs/config/agent/sample_agent.yaml", service="configs/service_functions/abc.yaml",
                  sim="configs/config/simulator/sample_config.yaml", episode_steps=200, period=10),
    "type4": dict(train=["configs/networks/Compuserve_n14_e17/Compuserve-in4-cap1.graphml",
                         "configs/networks/node6/node6-in2-cap1-delay10.graphml",
                         "configs/networks/Claranet_n15_e18/Claranet-in4-cap1.graphml"],
                  test="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml",
                  agent="configs/config/agent/sample_agent.yaml", service="configs/service_functions/abc.yaml",
                  sim="configs/config/simulator/sample_config.yaml", episode_steps=200, period=10),
    # diagnosis controls: one training network, tested on that same network (no transfer, no network switches)
    "solo_rc12": dict(train=["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                      test="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml",
                      agent="configs/config/agent/sample_agent.yaml", service="configs/service_functions/abc.yaml",
                      sim="configs/config/simulator/sample_config.yaml", episode_steps=200, period=10),
    "solo_cap1": dict(train=["configs/networks/abilene/abilene-in4-cap1.graphml"],
                      test="configs/networks/abilene/abilene-in4-cap1.graphml",
                      agent="configs/config/agent/sample_agent.yaml", service="configs/service_functions/abc.yaml",
                      sim="configs/config/simulator/sample_config.yaml", episode_steps=200, period=10),
    # 200-node: s0 / s1 for training (as bench config 5), s2 held out
    "syn200": dict(train=[f"{NET}/syn200-in16-cap1-3-s0.graphml", f"{NET}/syn200-in16-cap1-3-s1.graphml"],
                   test=f"{NET}/syn200-in16-cap1-3-s2.graphml", agent="configs/config/agent/agent_syn200.yaml",
                   service="configs/service_functions/abc-3sfc.yaml",
                   sim="configs/config/simulator/sample_config.yaml", episode_steps=20),
}


def uniform_rows(act, masks, topo, n_pad):
    """Fraction of the real schedule rows (source node of the topology) that post-processing left uniform over
    the real destinations -- the rows on which the schedule carries no information."""
    import torch
    E = act.shape[0]
    a = act.view(E, -1, n_pad)
    m = masks[topo].view(E, -1, n_pad) > 0
    real = m.any(-1)
    big = torch.where(m, a, torch.full_like(a, -1.0)).amax(-1)
    small = torch.where(m, a, torch.full_like(a, 2.0)).amin(-1)
    uni = (big - small).abs() < 1e-6
    return float((uni & real).sum()) / max(float(real.sum()), 1.0)


def evaluate(policy, cfg, net, pre, E, seed, learner=None, dev="cuda"):
    """Success ratio and mean return of ``policy`` over E test episodes (one per env) on topology ``net``.

    trained     greedy actor, post-processed like training actions (threshold / normalise)
    trained_raw greedy actor, raw weights (the reference's test path: no noise, no post-processing, Q7)
    noisy       actor + the training exploration noise, post-processed (the behaviour policy)
    random      uniform random weights per destination, post-processed (the warm-up policy)
    uniform     equal weights on every real destination"""
    import torch
    from gsc_amd.envs.common import schedule_threshold
    from gsc_amd.models.graphs import GraphSet
    from gsc_amd.native import load
    from gsc_amd.ops.explore import explore_postprocess
    from gsc_amd.sim.batched import load_batched_from_paths
    sim = load_batched_from_paths([net], pre["service"], pre["sim"], cfg, E, device=dev, seed=seed)
    obs = sim.reset().clone()
    graphs = GraphSet(sim.topologies, sim.n_pad, sim.device)
    masks = graphs.action_masks(sim.C, sim.F)
    thr = schedule_threshold(cfg, sim.n_pad)
    topo = torch.zeros(E, dtype=torch.int64, device=dev)
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    nat = load()
    uni = []
    sigma = float(cfg.get("rand_sigma", 0.3))
    for step in range(sim.episode_steps):
        pp = dict(seed=seed, step=step, topo=topo, threshold=thr)
        if policy in ("trained", "trained_raw", "noisy"):
            with learner._autocast(), torch.no_grad():
                mu = learner.actor(obs, topo, graphs, masks).float()
            if policy == "trained_raw":
                act = (mu * masks[topo]).contiguous()
            else:
                act = explore_postprocess(mu, masks, sim.n_pad, False, 0.0, sigma if policy == "noisy" else 0.0, **pp)
        elif policy == "random":
            mu = torch.zeros(E, sim.action_dim, device=dev)
            act = explore_postprocess(mu, masks, sim.n_pad, True, 0.0, 0.0, **dict(pp, seed=seed + 17))
        else:  # uniform: equal weights on the real destinations
            act = explore_postprocess(masks[topo].contiguous(), masks, sim.n_pad, False, 0.0, 0.0, **pp)
        uni.append(uniform_rows(act, masks, topo, sim.n_pad))
        out = sim.step(act, buffer_set=step & 1)
        st = out.stats
        nat.step_metrics(dev == "cuda", st.data_ptr(), st.shape[1], out.ep_return.data_ptr(), out.done.data_ptr(), E,
                         acc.data_ptr(), torch.cuda.current_stream().cuda_stream if dev == "cuda" else 0)
        obs = out.next_obs.clone()
    if dev == "cuda":
        torch.cuda.synchronize()
    sim.check_flags()
    s, d, r, e = [float(v) for v in acc.cpu()]
    return {"success_ratio": round(s / max(s + d, 1.0), 4), "episodes": int(e), "mean_return": round(r / max(e, 1.0), 3),
            "uniform_rows": round(sum(uni) / len(uni), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(PRESETS), default="syn50")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--train-steps", type=int, default=8000, help="lockstep steps of --envs envs")
    ap.add_argument("--eval-envs", type=int, default=64, help="test episodes on the held-out topology")
    ap.add_argument("--episode-steps", type=int, default=None)
    ap.add_argument("--schedule-threshold", default=None,
                    help="opt-in post-processing threshold (float or 'auto' = 2.4 / n_pad); default: the reference's 0.1")
    ap.add_argument("--on-train", action="store_true", help="also evaluate every policy on each training network")
    ap.add_argument("--check-every", type=int, default=0,
                    help="read the simulator's overflow / bad-state flags every N steps (0: at episode ends only)")
    a = ap.parse_args()
    import torch
    import yaml
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.sim.batched import load_batched_from_paths
    os.chdir(ROOT)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    pre = PRESETS[a.preset]
    cfg = yaml.safe_load(open(pre["agent"]))
    cfg["actor_output_activation"] = "sigmoid"
    cfg["episode_steps"] = int(a.episode_steps or pre["episode_steps"])
    if a.schedule_threshold is not None:
        cfg["schedule_threshold"] = a.schedule_threshold
    torch.manual_seed(a.seed)
    res = {"preset": a.preset, "seed": a.seed, "train": [os.path.basename(p) for p in pre["train"]],
           "test": os.path.basename(pre["test"]), "episode_steps": cfg["episode_steps"],
           "schedule_threshold": cfg.get("schedule_threshold", 0.1)}
    nets = [pre["test"]] + (list(pre["train"]) if a.on_train else [])
    evals = {os.path.basename(n): {} for n in nets}
    # baselines first (independent of training)
    for n in nets:
        for pol in ("random", "uniform"):
            evals[os.path.basename(n)][pol] = evaluate(pol, cfg, n, pre, a.eval_envs, 1000 + a.seed, dev=dev)
    sim = load_batched_from_paths(pre["train"], pre["service"], pre["sim"], cfg, a.envs, device=dev, seed=a.seed)
    T = len(pre["train"])
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=a.envs, seed=a.seed, check_every=a.check_every),
                        network_schedule=list(range(T)), period=int(pre.get("period", 1)))
    t0 = time.time()
    curve = []
    uni = []
    for step in range(a.train_steps):
        tr.step()
        if (step + 1) % cfg["episode_steps"] == 0 and step >= tr.learning_starts:  # explored, post-processed rows
            uni.append(uniform_rows(tr._act_bufs[step & 1], tr.masks, tr.topo, sim.n_pad))
        if (step + 1) % (cfg["episode_steps"] * 10) == 0:
            m = tr.metrics()
            curve.append(round(m["success_ratio"], 4))
            print(f"# {a.preset} seed {a.seed} step {step + 1} train success {m['success_ratio']:.4f} "
                  f"qf1 {m.get('qf1_loss', float('nan')):.4f} actor {m.get('actor_loss', float('nan')):.4g}",
                  flush=True)
    tr.flush()
    res["train_seconds"] = round(time.time() - t0, 1)
    res["train_env_steps"] = a.train_steps * a.envs
    res["train_curve_every_10_episodes"] = curve
    res["train_uniform_rows"] = round(sum(uni) / max(len(uni), 1), 4)
    for n in nets:
        for pol in ("trained", "trained_raw", "noisy"):
            evals[os.path.basename(n)][pol] = evaluate(pol, cfg, n, pre, a.eval_envs, 1000 + a.seed, learner=tr.learner,
                                                       dev=dev)
    res["eval"] = evals
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
