#!/usr/bin/env python
"""Micro-benchmark of the fused GATv2 embedder kernels (sample-agent shapes).

    python scripts/gnn_bench.py [--batch 25600] [--path 0|1|3] [--profile]

Times forward and forward+backward per call (HIP events); ``--profile`` prints the generic
backward's per-phase cycle counters (s_memtime, summed over waves, per graph).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["topo", "fwd-recompute", "bias", "d-alpha", "softmax-bwd", "d-att", "dxl/dxr", "dW", "d-bl/br|dh(cl)",
          "dh|relu-mask(cl)", "-", "-"]
MF_PHASES = ["topo+x", "fwd-recompute", "x_l/x_r", "bias+p+ssum", "scatter dX", "dX images", "dW mfma", "dh mfma",
             "-", "-", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=25600)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--path", type=int, default=None, help="bits: 1 cl fwd, 2 cl bwd, 4 node-lane fwd (0 = generic)")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--hidden", type=int, default=22)
    ap.add_argument("--network", default="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml")
    ap.add_argument("--n-pad", type=int, default=24)
    a = ap.parse_args()
    import torch
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GNNEmbedder, GraphSet
    from gsc_amd.native import load
    nat = load()
    if a.path is not None:
        nat.gnn_set_path(a.path)
    dev = "cuda"
    gs = GraphSet([load_topology(os.path.join(ROOT, a.network))], a.n_pad, dev)
    emb = GNNEmbedder(3, a.hidden, 2, "mean", 2).to(dev)
    B = a.batch
    topo = torch.zeros(B, dtype=torch.int64, device=dev)
    x = torch.rand(B, a.n_pad, 3, device=dev) * gs.node_mask[topo].unsqueeze(-1)
    w = torch.randn(a.hidden, device=dev)
    params = list(emb.parameters())

    def fwd():
        return emb(x, topo, gs, use_native=True)

    def fwdbwd():
        out = emb(x, topo, gs, use_native=True)
        return torch.autograd.grad((out * w).sum(), params)

    for f in (fwd, fwdbwd):
        f()
    torch.cuda.synchronize()
    res = {}
    for name, f in (("fwd", fwd), ("fwd+bwd", fwdbwd)):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            f()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / a.iters * 1e3
    print(f"path={nat.gnn_get_path()} B={B} fwd {res['fwd']:.1f} us  fwd+bwd {res['fwd+bwd']:.1f} us  "
          f"bwd~{res['fwd+bwd'] - res['fwd']:.1f} us")
    if a.profile:
        prof = torch.zeros(12, dtype=torch.int64, device=dev)
        nat.gnn_set_profile(prof.data_ptr())
        fwdbwd()
        torch.cuda.synchronize()
        nat.gnn_set_profile(0)
        p = prof.cpu().tolist()
        tot = sum(p)
        print("backward phase cycles per graph (s_memtime ticks, summed over waves; cl: bias+d-alpha in 'd-alpha'):")
        names = MF_PHASES if nat.gnn_get_path() & 32 else PHASES
        for k, v in enumerate(p):
            if v:
                print(f"  {names[k]:>14}: {v / B:10.1f}  ({100 * v / tot:5.1f} %)")


if __name__ == "__main__":
    main()
