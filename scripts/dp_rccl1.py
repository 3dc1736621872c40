#!/usr/bin/env python
"""The data-parallel learner path over a real RCCL communicator on ONE GPU (``GSC_DIST_FORCE=1``: a
world-size-1 ``nccl`` process group).

Every collective of the DP path is issued through RCCL: the parameter broadcast, the critic / actor-MLP /
actor-embedder gradient all-reduces captured inside the one HIP graph of ``update_graphed`` (and, with
``GSC_DP_GRAPH=0``, issued eagerly between five per-stage graphs), the ZeRO-1
reduce-scatter / all-gather and its guard agreement, and (with ``--bf16``) the bf16 gradient all-reduce.
With one rank every collective is an identity, so the result must equal the process-local learner
(one captured graph, no collectives) bit for bit.

Run:  GSC_DIST_FORCE=1 python scripts/dp_rccl1.py      -> one JSON line
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist
import yaml

from scripts.dp_rehearsal import batches, flats


def per_param(L):
    return {f"{net}.{k}": v.detach().clone() for net in ("actor", "critic", "target_actor", "target_critic")
            for k, v in getattr(L, net).state_dict().items()}


def main():
    from gsc_amd.agents import Batch, DDPGLearner
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GraphSet
    from gsc_amd.parallel.dist import init_distributed, shutdown

    assert os.environ.get("GSC_DIST_FORCE") == "1", "run with GSC_DIST_FORCE=1"
    info = init_distributed("cuda")
    dev = torch.device("cuda", torch.cuda.current_device())
    os.chdir(ROOT)
    cfg = yaml.safe_load(open("configs/config/agent/sample_agent.yaml"))
    net = "configs/networks/abilene/abilene-in4-rand-cap1-2.graphml"
    gs = GraphSet([load_topology(net)], 24, dev)
    B, n = 512, 4
    full = batches(n, B, dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(), "forced": info.forced}

    def run(dist_info, zero=False):
        L = DDPGLearner(cfg, 3, 1728, gs, 1, 3, dev, dist_info, seed=3, zero=zero)
        static = Batch(*(torch.empty_like(t) for t in full[0]))
        for b in full:
            for d, s in zip(static, b):
                d.copy_(s)
            L.update_graphed(static, warmup=1)
        torch.cuda.synchronize()
        return L

    ref = run(None)                       # process-local: one graph, no collectives
    res["ref_graphs"] = len(ref._graphs)
    D = run(info)                         # DP path over RCCL: all-reduces captured in the update graph
    res["dp_graphs"] = len(D._graphs)
    res["dp_bitwise"] = all(torch.equal(a, b) for a, b in zip(flats(D), flats(ref)))
    res["dp_grad_bitwise"] = (torch.equal(D.critic_flat.grad, ref.critic_flat.grad)
                              and torch.equal(D.actor_flat.grad, ref.actor_flat.grad))
    os.environ["GSC_DP_GRAPH"] = "0"      # fallback: five graphs, eager all-reduces between them
    E = run(info)
    os.environ.pop("GSC_DP_GRAPH")
    res["eager_graphs"] = len(E._graphs)
    res["eager_bitwise"] = all(torch.equal(a, b) for a, b in zip(flats(E), flats(ref)))
    Z = run(info, zero=True)              # ZeRO-1 over RCCL (reduce-scatter, Adam on the shard, all-gather)
    pz, pr = per_param(Z), per_param(ref)
    dz = torch.cat([(pz[k] - pr[k]).abs().view(-1) for k in pr])
    res["zero"] = bool(Z.zero)
    res["zero_bitwise"] = bool((dz == 0).all())
    res["zero_max_abs_diff"] = float(dz.max())
    os.environ["GSC_DP_GRAD_BF16"] = "1"  # bf16 gradient all-reduce: one rank rounds the gradient to bf16
    H = run(info)
    os.environ.pop("GSC_DP_GRAD_BF16")
    dh = torch.cat([(a - b).abs().view(-1) for a, b in zip(flats(H), flats(ref))])
    res["bf16"] = bool(H.grad_bf16)
    res["bf16_max_abs_diff"] = float(dh.max())
    print(json.dumps(res), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
