#!/usr/bin/env python
"""Data-parallel rehearsal on ONE GPU: N ranks (gloo collectives, GSC_DIST_BACKEND=gloo) through the
GPU learner's HIP-graph path (native kernels, 5 captured stages with the critic/actor gradient
all-reduces between them) and through the batched trainer (device simulator + learner).

Run:  GSC_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29511 scripts/dp_rehearsal.py

Rank 0 prints one JSON line:
  replicas_bitwise      every rank's four flat parameter buffers are bit-identical (all_gather + torch.equal)
  grad_vs_single        max relative error of the all-reduced critic / actor gradients of every update
                        against one process updating on the concatenated batch (same kernels, fp32
                        accumulation order); update 0 is the eager warm-up
  grad_vs_single_graphed  the same over the captured updates only (k >= 1: the five-stage graph path,
                        actor-MLP all-reduce overlapping the embedder backward)
  param_mismatch_frac   fraction of parameters differing by > 1e-4 from that single process after 3 updates
  trainer_replicas_bitwise  same check after 6 batched-trainer steps (per-rank envs, shared learner)
  zero_replicas_bitwise / zero_param_mismatch_frac  the sharded optimizer (ZeRO-1: reduce-scatter, Adam on
                        1/W, all-gather; gsc_amd/parallel/zero.py) on the native GPU kernels: replicas and
                        agreement with the single process after the same 3 updates
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist
import yaml


def flats(L):
    return [L.actor_flat.flat, L.critic_flat.flat, L.target_actor_flat.flat, L.target_critic_flat.flat]


def bitwise_same(tensors, world):
    ok = True
    for t in tensors:
        got = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(got, t.contiguous())
        ok &= all(torch.equal(got[0], g) for g in got[1:])
    return bool(ok)


def batches(n, B, dev):
    from gsc_amd.agents import Batch
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n):
        obs = torch.rand(B, 24, 3, generator=g)
        obs[:, 11:] = 0
        nxt = torch.rand(B, 24, 3, generator=g)
        nxt[:, 11:] = 0
        out.append(Batch(obs.to(dev), torch.zeros(B, dtype=torch.int64, device=dev),
                         torch.rand(B, 1728, generator=g).to(dev, torch.bfloat16),
                         (torch.rand(B, generator=g) - 0.5).to(dev), nxt.to(dev),
                         (torch.rand(B, generator=g) < 0.2).float().to(dev)))
    return out


def main():
    from gsc_amd.agents import Batch, BatchedTrainer, DDPGLearner, TrainerConfig
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GraphSet
    from gsc_amd.parallel.dist import init_distributed, shutdown
    from gsc_amd.sim.batched import load_batched_from_paths

    info = init_distributed("cuda")
    W, r = info.world_size, info.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    os.chdir(ROOT)
    cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
    net = "configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"
    gs = GraphSet([load_topology(net)], 24, dev)
    Bp = 512
    full = batches(3, Bp * W, dev)
    # (a) learner, HIP-graph path: ranks start from different seeds (rank 0's replicas are broadcast)
    L = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, info, seed=3 if r == 0 else 100 + r)
    assert L.native_ok
    static = Batch(*(torch.empty_like(t[:Bp]) for t in full[0]))
    grads = []
    for k, b in enumerate(full):
        for d, s in zip(static, b):
            d.copy_(s[r * Bp:(r + 1) * Bp])
        L.update_graphed(static, warmup=1)
        torch.cuda.synchronize()
        grads.append([L.critic_flat.grad.clone(), L.actor_flat.grad.clone()])   # all-reduced sums
    torch.cuda.synchronize()
    res = {"world": W, "backend": info.backend, "graphed": L._graphs is not None and len(L._graphs) == 5,
           "replicas_bitwise": bitwise_same(flats(L), W)}
    if r == 0:
        ref = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, None, seed=3)
        # single process: the same updates on the concatenated batches (world_size 1 inside the learner)
        per_k = []
        for k, b in enumerate(full):
            ref.update(b)
            torch.cuda.synchronize()
            # DP buffers hold the sum of per-rank means = W x the single-process mean gradient
            per_k.append(max(((g / W - rg).norm() / rg.norm()).item()
                             for g, rg in zip(grads[k], [ref.critic_flat.grad, ref.actor_flat.grad])))
        res["grad_vs_single"] = max(per_k)
        res["grad_vs_single_graphed"] = max(per_k[1:])
        torch.cuda.synchronize()
        d = torch.cat([(a - b).abs().view(-1) for a, b in zip(flats(L), flats(ref))])
        res["param_mismatch_frac"] = float((d > 1e-4).float().mean())
        res["param_max_abs_diff"] = float(d.max())
    # (c) sharded optimizer state (ZeRO-1) on the native kernels, same batches
    Z = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, info, seed=3 if r == 0 else 100 + r, zero=True)
    for k, b in enumerate(full):
        for d, s in zip(static, b):
            d.copy_(s[r * Bp:(r + 1) * Bp])
        Z.update_graphed(static, warmup=1)
    torch.cuda.synchronize()
    res["zero"] = bool(Z.zero)
    res["zero_moment_frac"] = Z.actor_opt.m.numel() / Z.actor_flat.flat.numel()
    res["zero_replicas_bitwise"] = bitwise_same(flats(Z), W)
    if r == 0:
        d = torch.cat([(getattr(Z, net).state_dict()[k] - v).abs().view(-1)
                       for net in ("actor", "critic", "target_actor", "target_critic")
                       for k, v in getattr(ref, net).state_dict().items()])
        res["zero_param_mismatch_frac"] = float((d > 1e-4).float().mean())
    # (b) batched trainer: per-rank envs, replicated learner, HIP-graph updates
    sim = load_batched_from_paths([net], "configs/service_functions/abc.yaml",
                                  "configs/config/simulator/sample_config.yaml", cfg, 32, device=dev, seed=1000 + r)
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=32, batch_size=256, learning_starts=2, seed=5 + 17 * r,
                                                check_every=0), info)
    for _ in range(6):
        tr.step()
    torch.cuda.synchronize()
    m = tr.metrics()
    res["trainer_replicas_bitwise"] = bitwise_same(flats(tr.learner), W)
    res["trainer_updates"] = tr.learner.updates
    res["trainer_graphed"] = tr.learner._graphs is not None
    res["envs_differ"] = not bitwise_same([sim.states], W)
    res["success_ratio"] = m["success_ratio"]
    if r == 0:
        print(json.dumps(res), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
