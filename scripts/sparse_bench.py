#!/usr/bin/env python
"""Standalone timing of the sparse replayed-action critic products (csrc/ops/sparse_act.hip) at config-5 scale.

Synthetic records (no trainer): B sampled transitions of R row blocks x P destinations, 5..11 exceptions per row at
spread indices, a uniform base on 20 % of the rows.  Times sparse_fwd (+ split-K reduction) and sparse_wgrad with
HIP events, optionally the dense bf16 GEMMs over the same [B, A] block for comparison (--dense).

    python scripts/sparse_bench.py --B 25600 --R 1800 --P 200 --iters 10 [--dense]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gsc_amd.agents.native_update import sparse_fwd_splits  # noqa: E402
from gsc_amd.native import load  # noqa: E402


def records(B, R, P, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = B * R
    rec = torch.zeros(n, 12, dtype=torch.int32, device="cuda")
    cnt = torch.randint(5, 12, (n,), device="cuda", generator=g)
    uni = torch.rand(n, device="cuda", generator=g) < 0.2
    base = torch.where(uni, torch.full((n,), 1.0 / P, device="cuda"), torch.zeros(n, device="cuda"))
    b16 = base.to(torch.bfloat16).view(torch.int16).to(torch.int32) & 0xffff
    rec[:, 0] = b16 | (cnt << 16)
    step = P // 11
    k = torch.arange(11, device="cuda")
    idx = k * step + torch.randint(0, step, (n, 11), device="cuda", generator=g)
    val = (torch.rand(n, 11, device="cuda", generator=g) * 0.5).to(torch.bfloat16).view(torch.int16).to(torch.int32)
    slots = (idx & 0xffff) | ((val & 0xffff) << 16)
    slots = torch.where(k[None, :] < cnt[:, None], slots, torch.zeros_like(slots))
    rec[:, 1:] = slots
    return rec.view(B, R, 12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=25600)
    ap.add_argument("--R", type=int, default=1800)
    ap.add_argument("--P", type=int, default=200)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--dense", action="store_true")
    a = ap.parse_args()
    nat = load()
    B, R, P, c1 = a.B, a.R, a.P, 64
    A = R * P
    ring = records(B, R, P)
    rows = torch.randperm(B, device="cuda").to(torch.int32)
    lda = (A + 7) // 8 * 8
    wa = (torch.randn(c1, lda, device="cuda") * 0.05).to(torch.bfloat16)
    dh0 = torch.randn(B, c1, device="cuda").to(torch.bfloat16)
    S = a.splits or sparse_fwd_splits(B, R, 64, torch.device("cuda"))
    part = torch.empty(S, B, c1, device="cuda")
    wsum = torch.empty(R * c1, dtype=torch.int32, device="cuda")
    hacc = torch.empty(B, c1, device="cuda")
    gw = torch.empty(c1, A, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def fwd():
        nat.sparse_fwd(ring.data_ptr(), rows.data_ptr(), B, R, P, wa.data_ptr(), lda, c1, wsum.data_ptr(), part.data_ptr(), S, s)
        nat.splitk_reduce(part.data_ptr(), B * c1, S, B, c1, c1, hacc.data_ptr(), c1, 1.0, 0, s)

    def wgrad():
        nat.sparse_wgrad(ring.data_ptr(), rows.data_ptr(), B, R, P, dh0.data_ptr(), c1, c1, gw.data_ptr(), A, s)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    flop = 2.0 * B * A * c1
    tf, tg = timeit(fwd), timeit(wgrad)
    print(f"B={B} R={R} P={P} splits={S} sparse_fwd+reduce {tf:.3f} ms ({flop / tf / 1e9:.0f} TFLOP/s)  "
          f"sparse_wgrad {tg:.3f} ms ({flop / tg / 1e9:.0f} TFLOP/s)", flush=True)
    if a.dense:
        from gsc_amd.ops.mlp import gemm
        dense = torch.empty(B, lda, dtype=torch.bfloat16, device="cuda")
        dense.zero_()
        slabs = torch.empty(64 * B * c1, device="cuda")
        h2 = torch.empty(B, c1, device="cuda")
        td = timeit(lambda: gemm(dense[:, :A], wa[:, :A], "nt", out32=h2, splits=None, slabs=slabs))
        tdg = timeit(lambda: gemm(dh0, dense[:, :A], "tn", out32=gw, splits=None, slabs=slabs))
        print(f"dense fwd {td:.3f} ms  dense wgrad {tdg:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
