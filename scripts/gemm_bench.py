#!/usr/bin/env python
"""Skinny bf16 GEMM formulations of the critic's action projection ([B, A] x [A, h])."""
import torch
import torch.nn.functional as F


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for B, A, h in ((25600, 1728, 64), (25600, 1728, 256), (25600, 256, 1728), (25600, 64, 1728)):
    x = torch.randn(B, A, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(h, A, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(B, h, device="cuda", dtype=torch.bfloat16)
    r = {
        "linear x W^T": t(lambda: F.linear(x, w)),
        "(W x^T)^T": t(lambda: torch.mm(w, x.t()).t()),
        "dW = g^T x": t(lambda: torch.mm(g.t(), x)),
        "dW via (x^T g)^T": t(lambda: torch.mm(x.t(), g).t()),
        "dX = g W": t(lambda: torch.mm(g, w)),
    }
    gb = (B * A + A * h + B * h) * 2 / 1e9
    print(f"B={B} A={A} h={h} ({gb * 1e3:.0f} MB min traffic, {gb / 5e3 * 1e6:.0f} us @5TB/s): " +
          "  ".join(f"{k} {v:.1f}us" for k, v in r.items()), flush=True)

print("split-K weight gradients (bmm over K-chunks + fp32 sum):")
for B, A, h in ((25600, 1728, 64), (25600, 22, 64), (25600, 22, 256), (25600, 256, 64)):
    x = torch.randn(B, A, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(B, h, device="cuda", dtype=torch.bfloat16)
    ref = torch.mm(g.t().float(), x.float())
    res = {"mm": t(lambda: torch.mm(g.t(), x))}
    for C in (8, 16, 32, 64):
        if B % C:
            continue
        def f(C=C):
            p = torch.bmm(g.view(C, B // C, h).transpose(1, 2), x.view(C, B // C, A))
            return p.float().sum(0)
        err = (f() - ref).abs().max().item() / ref.abs().max().item()
        res[f"C={C}"] = t(f)
        res[f"C={C}_err"] = err
    print(f"  dW [{h}x{A}] K={B}: " + "  ".join(f"{k} {v:.3g}" for k, v in res.items()), flush=True)
