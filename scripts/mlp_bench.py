"""Time the MFMA GEMM engine on the DDPG learner's shapes (Abilene, batch 25,600) vs hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gsc_amd.ops.mlp import gemm


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


B, A, H1, C1 = 25600, 1728, 256, 64
d = "cuda"
bf = torch.bfloat16
z = torch.randn(B, H1, device=d, dtype=bf)
w2 = torch.randn(A, H1, device=d, dtype=bf)
act = torch.randn(B, A, device=d, dtype=bf)
wca = torch.randn(C1, A, device=d, dtype=bf)
dh = torch.randn(B, C1, device=d, dtype=bf)
o_a = torch.empty(B, A, device=d, dtype=bf)
o_h = torch.empty(B, C1, device=d)
o_w = torch.empty(C1, A, device=d)
o_w2 = torch.empty(A, H1, device=d)
slabs = torch.empty(32 * A * H1, device=d)
rows = []
for tile in (0, 1, 2):
    rows.append((f"z@W2^T [B,256]x[256,1728] tile{tile}", bench(lambda: gemm(z, w2, "nt", out16=o_a, tile=tile)),
                 bench(lambda: torch.mm(z, w2.t()))))
for tile in (1, 2):
    rows.append((f"a@Wca^T [B,1728]x[1728,64] tile{tile}", bench(lambda: gemm(act, wca, "nt", out32=o_h, tile=tile)),
                 bench(lambda: torch.mm(act, wca.t()))))
for sp in (8, 16, 32):
    rows.append((f"dh^T a [64,B]x[B,1728] split{sp}",
                 bench(lambda: gemm(dh, act, "tn", out32=o_w, splits=sp, slabs=slabs)),
                 bench(lambda: torch.mm(dh.t(), act))))
    rows.append((f"da^T z [1728,B]x[B,256] split{sp}",
                 bench(lambda: gemm(act, z, "tn", out32=o_w2, splits=sp, slabs=slabs)),
                 bench(lambda: torch.mm(act.t(), z))))
rows.append(("dh@Wca [B,64]x[64,1728] nn", bench(lambda: gemm(dh, wca, "nn", out16=o_a)),
             bench(lambda: torch.mm(dh, wca))))
rows.append(("da@W2 [B,1728]x[1728,256] nn", bench(lambda: gemm(act, w2, "nn", out16=z)),
             bench(lambda: torch.mm(act, w2))))
print(f"{'shape':45s} {'mfma us':>9s} {'torch us':>9s}")
for n, a, b in rows:
    print(f"{n:45s} {a:9.1f} {b:9.1f}")
