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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=256, help="environments per GPU")
    ap.add_argument("--batch-size", type=int, default=None, help="learner batch (default 100 * envs)")
    ap.add_argument("--updates-per-step", type=int, default=1)
    ap.add_argument("--network", default="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml")
    ap.add_argument("--service", default="configs/service_functions/abc.yaml")
    ap.add_argument("--sim-config", default="configs/config/simulator/sample_config.yaml")
    ap.add_argument("--agent-config", default="configs/config/agent/sample_agent.yaml")
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

    device_type = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    info = init_distributed(device_type)
    if device_type == "cuda":
        dev_index = info.local_rank % torch.cuda.device_count()
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    os.chdir(ROOT)
    cfg = yaml.safe_load(open(args.agent_config))
    sim = load_batched_from_paths([args.network], args.service, args.sim_config, cfg, args.envs, device=device,
                                  seed=args.seed * 1000 + info.rank)
    tcfg = TrainerConfig(num_envs=args.envs, batch_size=args.batch_size, updates_per_step=args.updates_per_step,
                         learning_starts=1, seed=args.seed + 17 * info.rank, check_every=0,
                         overlap_sim=not args.no_overlap, sim_cus=args.sim_cus)
    trainer = BatchedTrainer(cfg, sim, tcfg, info)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        trainer.step()
    sync()
    trainer.metrics(reset=True)
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    sync()
    barrier()
    dt = time.perf_counter() - t0
    sim.check_flags()
    m = trainer.metrics(reset=True)

    if args.check_replicas and info.enabled:
        import torch.distributed as dist
        L = trainer.learner
        sig = torch.stack([t.double().sum() for t in (L.actor_flat.flat, L.critic_flat.flat, L.target_actor_flat.flat,
                                                      L.target_critic_flat.flat)])
        sigs = [torch.zeros_like(sig) for _ in range(info.world_size)]
        dist.all_gather(sigs, sig)
        same = all(torch.equal(sigs[0], x) for x in sigs)
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
    if info.is_main:
        rec = {
            "metric": "env-steps/sec (whole node) + flow success ratio, Abilene SFC",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": info.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_ENV_STEPS_PER_S, 1),
            "dtype": "bf16" if device.type == "cuda" else "fp32",
            "data": "synthetic (coord-sim sample_config traffic on Abilene-in4-rand-cap1-2, abc SFC), random-init weights",
            "success_ratio": round(m["success_ratio"], 4),
            "config": {
                "model": "GSC GATv2-DDPG (GNN 22x2L2I, actor [256] 893,628 params, critic [64] 223,997 params)",
                "global_batch": trainer.batch_size * info.world_size,
                "seq_len": sim.episode_steps,
                "parallelism": f"dp{info.world_size}",
                "envs_per_gpu": args.envs,
                "total_envs": total_envs,
                "learner_batch_per_gpu": trainer.batch_size,
                "updates_per_step": args.updates_per_step,
                "sim_learner_overlap": not args.no_overlap,
                "sim_cus": getattr(trainer, "sim_cus", 0),
                "topology": os.path.basename(args.network),
                "device": torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu",
            },
        }
        print(json.dumps(rec), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
