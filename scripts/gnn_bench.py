#!/usr/bin/env python
"""Micro-benchmark of the native GATv2 embedder kernels (sample-agent shapes, default routing:
MFMA one-tile <= 32 nodes, two-tile 33..64 nodes, layer-wise beyond).

    python scripts/gnn_bench.py [--batch 25600] [--network <graphml>] [--n-pad 24]

Times the inference forward, the grad-requiring forward (saves the per-layer state) and
forward+backward per call (HIP events).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=25600)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hidden", type=int, default=22)
    ap.add_argument("--network", default="configs/networks/abilene/abilene-in4-rand-cap1-2.graphml")
    ap.add_argument("--n-pad", type=int, default=24)
    a = ap.parse_args()
    import torch
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GNNEmbedder, GraphSet
    from gsc_amd.ops.gnn import gnn_use_fused
    dev = "cuda"
    gs = GraphSet([load_topology(os.path.join(ROOT, a.network))], a.n_pad, dev)
    emb = GNNEmbedder(3, a.hidden, 2, "mean", 2).to(dev)
    B = a.batch
    topo = torch.zeros(B, dtype=torch.int64, device=dev)
    x = torch.rand(B, a.n_pad, 3, device=dev) * gs.node_mask[topo].unsqueeze(-1)
    w = torch.randn(a.hidden, device=dev)
    params = list(emb.parameters())

    def fwd():
        with torch.no_grad():
            return emb(x, topo, gs, use_native=True)

    def fwd_save():
        return emb(x, topo, gs, use_native=True)

    def fwdbwd():
        out = emb(x, topo, gs, use_native=True)
        return torch.autograd.grad((out * w).sum(), params)

    for f in (fwd, fwd_save, fwdbwd):
        f()
    torch.cuda.synchronize()
    res = {}
    for name, f in (("fwd", fwd), ("fwd_save", fwd_save), ("fwd+bwd", fwdbwd)):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            f()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / a.iters * 1e3
    kind = "fused-mfma" if gnn_use_fused(emb, gs, a.n_pad, 3) else "layer-wise"
    print(f"{os.path.basename(a.network)} nodes={gs.max_nodes} n_pad={a.n_pad} {kind} B={B}: "
          f"fwd {res['fwd']:.1f} us  fwd(save) {res['fwd_save']:.1f} us  fwd+bwd {res['fwd+bwd']:.1f} us  "
          f"bwd~{res['fwd+bwd'] - res['fwd_save']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
