#!/usr/bin/env python
"""Time the MFMA GEMM engine (csrc/ops/mlp.hip) at the DDPG learner's shapes for every output tile x
K-stage depth, next to hipBLASLt (torch.mm) as a yardstick.

    python scripts/gemm_tune.py [abilene|syn200] [B]

abilene: B = 25,600, A = 1,728 (sample agent); syn200: A = 360,000, 3 topologies (config 5), B = 25,600 (the
preset's 100 samples per env-step at 256 envs) unless given."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from gsc_amd.ops.mlp import gemm


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


PRESET = sys.argv[1] if len(sys.argv) > 1 else "abilene"
dev = "cuda"
bf = torch.bfloat16
if PRESET == "abilene":
    B = 25600
    cases = [  # (name, layout, a, b, kwargs)
        ("actor out  [B,256]x[1728,256]^T -> bf16", "nt", (B, 256), (1728, 256), {}),
        ("critic act [B,1728]x[64,1728]^T -> f32", "nt", (B, 1728), (64, 1728), {"o32": True}),
        ("critic dW  [B,64]^T x [B,1728]", "tn", (B, 64), (B, 1728), {"o32": True, "split": True}),
        ("actor hid  [B,22]x[256,22]^T -> bf16", "nt", (B, 22), (256, 22), {}),
        ("dX  [B,64]x[64,256] -> bf16", "nn", (B, 64), (64, 256), {}),
    ]
else:
    B, A, T = int(sys.argv[2]) if len(sys.argv) > 2 else 25600, 360000, 3
    cases = [
        ("target actor out [B,256]x[A,256]^T -> bf16 (masked, clamped)", "nt", (B, 256), (A, 256), {"mask": True}),
        ("critic act [B,A]x[64,A]^T -> f32 (split-K)", "nt", (B, A), (64, A), {"o32": True, "split": True}),
        ("critic dW  [B,64]^T x [B,A]", "tn", (B, 64), (B, A), {"o32": True, "split": True}),
        ("Mc  [3*64,A]x[A,256] -> f32 (split-K)", "nn", (T * 64, A), (A, 256), {"o32": True, "split": True}),
        ("actor dW  [3*64,A]^T x [3*64,256]", "tn", (T * 64, A), (T * 64, 256), {"o32": True}),
    ]
    masks = (torch.rand(T, A, device=dev) > 0.5).float()
    topo = torch.randint(0, T, (B,), device=dev, dtype=torch.int32)
slabs = torch.empty(16 << 20, device=dev)
if PRESET != "abilene":   # the TD target's actor output + critic projection: materialised vs fused
    from gsc_amd.native import load as load_native
    nat = load_native()
    h = torch.randn(B, 256, device=dev, dtype=bf)
    w = torch.randn(A, 256, device=dev, dtype=bf) * 0.05
    bias = torch.zeros(A, device=dev)
    wa = torch.randn(64, A, device=dev, dtype=bf) * 0.05
    act = torch.empty(B, A, device=dev, dtype=bf)
    z = torch.empty(B, 64, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def materialised():
        gemm(h, w, "nt", out16=act, bias=bias, colmask=masks, topo=topo, clamp=(-1.0, 1.0), tile=1)
        gemm(act, wa, "nt", out32=z, splits=None, slabs=slabs, tile=1)

    def fused():
        nat.actor_proj(h.data_ptr(), 256, w.data_ptr(), 256, bias.data_ptr(), masks.data_ptr(), A, T, topo.data_ptr(),
                       wa.data_ptr(), A, B, 256, A, 64, -1.0, 1.0, slabs.data_ptr(), slabs.numel(), z.data_ptr(), 64, st)
    print(f"TD-target projection [B,256] -> [B,A] -> [B,64]: materialised {t(materialised):.1f} us  "
          f"fused {t(fused):.1f} us", flush=True)
for name, lay, sa, sb, kw in cases:
    a = torch.randn(*sa, device=dev, dtype=bf)
    b = torch.randn(*sb, device=dev, dtype=bf)
    if lay == "nt":
        M, N = sa[0], sb[0]
    elif lay == "tn":
        M, N = sa[1], sb[1]
    else:
        M, N = sa[0], sb[1]
    o16 = torch.empty(M, N, device=dev, dtype=bf)
    o32 = torch.empty(M, N, device=dev)
    res = {}
    for tile in (0, 1, 2, 3):
        for bk in (32, 64):
            ep = dict(colmask=masks, topo=topo, clamp=(-1.0, 1.0)) if kw.get("mask") else {}
            f = lambda: gemm(a, b, lay, out16=None if kw.get("o32") else o16, out32=o32 if kw.get("o32") else None,
                             tile=tile, bk=bk, splits=None if kw.get("split") else 1, slabs=slabs, **ep)
            res[f"t{tile}/bk{bk}"] = t(f)
    ref = {"nt": lambda: torch.mm(a, b.t()), "tn": lambda: torch.mm(a.t(), b), "nn": lambda: torch.mm(a, b)}[lay]
    res["hipblaslt"] = t(ref)
    best = min((v, k) for k, v in res.items() if k != "hipblaslt")
    print(f"{name}: " + "  ".join(f"{k} {v:.1f}" for k, v in res.items()) + f"  | best {best[1]} {best[0]:.1f} us",
          flush=True)
