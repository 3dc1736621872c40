#!/usr/bin/env python
"""Flagship benchmark: end-to-end GATv2-DDPG training throughput on the batched simulator.

Metric (BASELINE.json): env-steps/sec for the whole node + flow success ratio, Abilene SFC.
Config: Abilene-in4-rand-cap1-2 + ``abc`` SFC + ``sample_config`` traffic, reference model
(``sample_agent.yaml``: GNN 22x(2 layers, 2 iters), actor [256], critic [64]; actor 893,628 /
critic 223,997 parameters), E environments per GPU (default 256), bf16 GEMMs with fp32 master
weights.  One timed step = every env takes one 100 ms simulator step (actor forward, exploration +
post-processing, simulator kernel, replay insert) + ``updates_per_step`` DDPG updates on
``batch_size`` replayed transitions (default 100 per env step, the reference's ratio of gradient
samples to environment steps).  Weak scaling: E envs per GPU.

Run: ``python bench.py --gpus 1 --steps 50 --warmup 10``; multi-GPU via
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_ENV_STEPS_PER_S = 57.4  # reference env-only throughput, Abilene + abc, 1 CPU core

PRESETS = {
    "line": dict(network=["configs/networks/line/line4-in1-cap1-delay10.graphml"],
                 service="configs/service_functions/abc.yaml",
                 sim_config="configs/config/simulator/sample_config.yaml",
                 agent_config="configs/config/agent/sample_agent_flat.yaml", envs=1, batch=100, period=0,
                 device="cpu",
                 model="flat 2-layer MLP DDPG (graph_mode: False, actor/critic [64, 64]), 4-node line, 1 SFC (3 SFs)"),
    "abilene": dict(network=["configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"],
                    service="configs/service_functions/abc.yaml",
                    sim_config="configs/config/simulator/sample_config.yaml",
                    agent_config="configs/config/agent/sample_agent.yaml", envs=256, batch=None, period=0,
                    model="GSC GATv2-DDPG (GNN 22x2L2I, actor [256] 893,628 params, critic [64] 223,997 params)"),
    "syn50": dict(network=["configs/networks/synthetic/syn50-in8-cap1-3.graphml"],
                  service="configs/service_functions/abc-3sfc.yaml",
                  sim_config="configs/config/simulator/rand-arrival12_trace_syn50.yaml",
                  agent_config="configs/config/agent/agent_syn50.yaml", envs=256, batch=None, period=0,
                  model="GSC GATv2-DDPG, 50-node synthetic topology, 3 SFCs, trace traffic (A = 22,500)"),
    # BASELINE config 5 ("scheduler-driven network changes during training"): the network scheduler
    # switches every env to the next topology at every episode end (period 1) and episodes are 20 steps,
    # so any timed window of more than 20 steps contains a switch (counted in the JSON line).  256 envs and
    # the common learner ratio (100 replayed samples per env-step: B = 25,600); the [B, A] action blocks
    # are never materialised (replay rows read in place by the critic GEMM, composed actor loss, fused
    # TD-target projection), so A = 360,000 costs HBM bandwidth, not capacity
    "syn200": dict(network=[f"configs/networks/synthetic/syn200-in16-cap1-3-s{i}.graphml" for i in range(3)],
                   service="configs/service_functions/abc-3sfc.yaml",
                   sim_config="configs/config/simulator/sample_config.yaml",
                   agent_config="configs/config/agent/agent_syn200.yaml", envs=256, batch=None, period=1,
                   episode_steps=20,
                   model="GSC GATv2-DDPG, 200-node synthetic topologies switched every episode (20 steps), 3 SFCs "
                         "(A = 360,000)"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=None, help="environments per GPU (preset default: 256)")
    ap.add_argument("--batch-size", type=int, default=None, help="learner batch (default 100 * envs)")
    ap.add_argument("--updates-per-step", type=int, default=1)
    ap.add_argument("--preset", choices=sorted(PRESETS), default="abilene",
                    help="abilene: BASELINE configs 2/3 (headline); line: config 1 (4-node line, flat MLP, 1 CPU env); "
                         "syn50: config 4 (50-node + 3 SFCs + trace); "
                         "syn200: config 5 (200-node topologies switched by the network scheduler)")
    ap.add_argument("--network", default=None, help="override the preset's network(s) (comma-separated)")
    ap.add_argument("--service", default=None)
    ap.add_argument("--sim-config", default=None)
    ap.add_argument("--agent-config", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-overlap", action="store_true", help="run the simulator on the learner's stream")
    ap.add_argument("--check-replicas", action="store_true",
                    help="after timing, verify that every rank holds bit-identical parameters")
    ap.add_argument("--sim-cus", type=int, default=-1,
                    help="CUs reserved for the simulator stream (contiguous CU-mask bits); 0 = shared CUs, "
                         "-1 = auto (one round of env workgroups)")
    args = ap.parse_args()

    import torch
    import yaml

    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.parallel.dist import barrier, init_distributed, shutdown
    from gsc_amd.sim.batched import load_batched_from_paths

    pre = PRESETS[args.preset]
    networks = args.network.split(",") if args.network else pre["network"]
    service = args.service or pre["service"]
    sim_config = args.sim_config or pre["sim_config"]
    agent_config = args.agent_config or pre["agent_config"]
    if args.envs is None:
        args.envs = pre["envs"]
    if args.batch_size is None:
        args.batch_size = pre["batch"]
    device_type = args.device or pre.get("device") or ("cuda" if torch.cuda.is_available() else "cpu")
    info = init_distributed(device_type)
    if device_type == "cuda":
        dev_index = info.local_rank % torch.cuda.device_count()
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    os.chdir(ROOT)
    cfg = yaml.safe_load(open(agent_config))
    if pre.get("episode_steps"):
        cfg["episode_steps"] = int(pre["episode_steps"])
    sim = load_batched_from_paths(networks, service, sim_config, cfg, args.envs, device=device,
                                  seed=args.seed * 1000 + info.rank)
    tcfg = TrainerConfig(num_envs=args.envs, batch_size=args.batch_size, updates_per_step=args.updates_per_step,
                         learning_starts=1, seed=args.seed + 17 * info.rank, check_every=0,
                         overlap_sim=not args.no_overlap, sim_cus=args.sim_cus, lazy_handoff=True)
    trainer = BatchedTrainer(cfg, sim, tcfg, info, network_schedule=list(range(len(networks))),
                             period=pre["period"])

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        trainer.step()
    sync()
    trainer.metrics(reset=True)
    # diagnostics only (GSC_SIM_PROFILE=1, never for reported numbers): the simulator runs its cycle-counting
    # variant and the effective engine clock while it runs beside the learner is printed to stderr
    diag = os.environ.get("GSC_SIM_PROFILE") == "1" and device.type == "cuda"
    if diag:
        sim.enable_profiling()
    # GSC_PROF_WINDOW=1: one roctx range around exactly the timed steps, so a
    # `rocprofv3 --kernel-trace --marker-trace` table can be cut to the timed region (scripts/prof_summary.py)
    window = os.environ.get("GSC_PROF_WINDOW") == "1" and device.type == "cuda"
    barrier()
    sync()
    if window:
        torch.cuda.nvtx.range_push("bench_timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    sync()
    if window:
        torch.cuda.nvtx.range_pop()
    barrier()
    dt = time.perf_counter() - t0
    sim.check_flags()
    m = trainer.metrics(reset=True)
    if diag:
        ty = sim.prof[sim.E * 4:].view(sim.E, 64, 2).sum(0).double().cpu()
        ph = {k: ty[i, 0] / max(float(ty[i, 1]), 1) for k, i in (("copy_in", 60), ("copy_out", 61), ("prologue", 62),
                                                                  ("epilogue", 63))}
        print(f"diag: sim cycles/env-step={ty[58, 0] / max(float(ty[58, 1]), 1):.0f} "
              f"effective engine clock {ty[58, 0] / max(float(ty[59, 0]), 1) * 100:.0f} MHz "
              + " ".join(f"{k}={v:.0f}" for k, v in ph.items()), file=sys.stderr)

    if args.check_replicas and info.enabled:
        import torch.distributed as dist
        L = trainer.learner
        same = True
        for t in (L.actor_flat.flat, L.critic_flat.flat, L.target_actor_flat.flat, L.target_critic_flat.flat):
            got = [torch.empty_like(t) for _ in range(info.world_size)]
            dist.all_gather(got, t)
            same &= all(torch.equal(got[0], x) for x in got[1:])   # bitwise
        if info.is_main:
            print(json.dumps({"replicas_identical": bool(same), "updates": L.updates,
                              "graphed": bool(L._graphs is not None)}), flush=True)
        assert same, "parameter replicas diverged across ranks"
    dt_t = torch.tensor([dt], dtype=torch.float64, device=device)
    if info.enabled:
        import torch.distributed as dist
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_envs = args.envs * info.world_size
    value = total_envs * args.steps / dt
    # topology switches of the network scheduler inside the timed window (episode ends at steps
    # k * episode_steps - 1; the episode that starts after one uses schedule[(episode // period) % T])
    ep_steps, T = sim.episode_steps, len(networks)
    period = pre["period"]
    switches = 0
    if period and T > 1:
        topo_of = lambda ep: (ep // period) % T
        for ep in range(args.warmup // ep_steps + 1, (args.warmup + args.steps) // ep_steps + 1):
            if ep * ep_steps < args.warmup + args.steps and topo_of(ep) != topo_of(ep - 1):
                switches += 1
    if info.is_main:
        rec = {
            "metric": "env-steps/sec (whole node) + flow success ratio, Abilene SFC" if args.preset == "abilene"
            else f"env-steps/sec (whole node) + flow success ratio, {args.preset} (BASELINE config "
                 f"{ {'line': '1', 'syn50': '4', 'syn200': '5'}[args.preset] })",
            "value": float(f"{value:.6g}"),
            "unit": "env-steps/s",
            "n_gpus": info.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": float(f"{dt / args.steps * 1e3:.6g}"),
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.md quotes the reference only on Abilene; the synthetic presets have no baseline
            "vs_baseline": round(value / BASELINE_ENV_STEPS_PER_S, 1) if args.preset == "abilene" else None,
            "dtype": "bf16" if device.type == "cuda" else "fp32",
            "data": (f"synthetic (coord-sim {os.path.basename(sim_config)} traffic on "
                     f"{', '.join(os.path.basename(n) for n in networks)}, {os.path.basename(service)}), "
                     "random-init weights"),
            "success_ratio": round(m["success_ratio"], 4),
            **({"diagnostic": "GSC_SIM_PROFILE=1: cycle-counting simulator variant, not a benchmark number"}
               if diag else {}),
            "config": {
                "model": pre["model"],
                "global_batch": trainer.batch_size * info.world_size,
                "seq_len": sim.episode_steps,
                "parallelism": f"dp{info.world_size}",
                **({"dist_forced": True, "dist_backend": info.backend} if info.forced else {}),
                "envs_per_gpu": args.envs,
                "total_envs": total_envs,
                "learner_batch_per_gpu": trainer.batch_size,
                "updates_per_step": args.updates_per_step,
                "sim_learner_overlap": not args.no_overlap,
                "sim_cus": getattr(trainer, "sim_cus", 0),
                "episode_steps": ep_steps,
                "replay_capacity": trainer.replay.capacity,
                "replay_actions": "sparse rows" if getattr(trainer.replay, "sparse_rows", 0) else "dense",
                **({"peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 1)}
                   if device.type == "cuda" else {}),
                "scheduler_period": period,
                "topology_switches_timed": switches,
                "topology": ",".join(os.path.basename(n) for n in networks),
                "device": torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu",
            },
        }
        print(json.dumps(rec), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
