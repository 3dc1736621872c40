#!/usr/bin/env python
"""Exploration + post-processing kernel timing at a bench preset's action shape (no simulator).

E envs x A = n_pad^2 C F weights, mu uniform in [0, 1) (a sigmoid actor's range), one topology mask table, and
optionally the simulator's destination bitsets (``--pmask``: written into a scratch buffer of the simulator's
layout).  Times ``--iters`` launches with HIP events, noisy (non-warm-up) and warm-up.

    python scripts/explore_bench.py --n-pad 200 --envs 256 --pmask
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-pad", type=int, default=200)
    ap.add_argument("--nodes", type=int, default=None, help="real nodes (default n_pad)")
    ap.add_argument("--C", type=int, default=3)
    ap.add_argument("--F", type=int, default=3)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pmask", action="store_true")
    a = ap.parse_args()
    import torch
    from gsc_amd.ops.explore import explore_postprocess
    P, n, E = a.n_pad, a.nodes or a.n_pad, a.envs
    A = P * P * a.C * a.F
    m = torch.zeros(1, P, a.C, a.F, P, device="cuda")
    m[:, :n, :, :, :n] = 1
    mask = m.view(1, A)
    topo = torch.zeros(E, dtype=torch.int64, device="cuda")
    mu = torch.rand(E, A, device="cuda") * mask
    out = torch.empty(E, A, device="cuda")
    pm = None
    if a.pmask:
        stride = P * a.C * a.F * 32
        buf = torch.zeros(E * stride, dtype=torch.uint8, device="cuda")
        pm = (buf.data_ptr(), stride, a.C, a.F, a.C, a.F, P)
    gbytes = 2 * E * A * 4 / 1e9

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    # the same bytes moved by the copy engine-free PyTorch kernels: the practical roofline of this pattern
    us = timed(lambda: out.copy_(mu))
    print(f"copy  mu -> out (read + write {gbytes:.2f} GB): {us:.1f} us ({gbytes / (us * 1e-6):.0f} GB/s)", flush=True)
    us = timed(lambda: out.fill_(0.5))
    print(f"fill  out (write {gbytes / 2:.2f} GB): {us:.1f} us ({gbytes / 2 / (us * 1e-6):.0f} GB/s)", flush=True)
    for warm in (False, True):
        for i in range(3):
            explore_postprocess(mu, mask, P, warm, 0.0, 0.3, seed=1, step=i, out=out, topo=topo, pmask=pm)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            explore_postprocess(mu, mask, P, warm, 0.0, 0.3, seed=1, step=i, out=out, topo=topo, pmask=pm)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(f"explore P={P} n={n} E={E} A={A} warmup={int(warm)} pmask={int(a.pmask)}: {us:.1f} us "
              f"({gbytes / (us * 1e-6):.0f} GB/s for mu read + out write)", flush=True)


if __name__ == "__main__":
    main()
