"""Where the large-N GEMM time goes: [2048,256] x [360000,256]^T with different epilogues."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from gsc_amd.ops.mlp import gemm  # noqa: E402


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


B, A, T, K = 2048, 360000, 3, 256
dev = "cuda"
a = torch.randn(B, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(A, K, device=dev, dtype=torch.bfloat16)
o16 = torch.empty(B, A, device=dev, dtype=torch.bfloat16)
o32 = torch.empty(B, A, device=dev)
masks = (torch.rand(T, A, device=dev) > 0.5).float()
topo = torch.randint(0, T, (B,), device=dev, dtype=torch.int32)
m1 = masks[:1].contiguous()
for tile in (1, 2):
    for name, kw in (("bf16 plain", dict(out16=o16)), ("fp32 plain", dict(out32=o32)),
                     ("bf16 colmask 1 topo", dict(out16=o16, colmask=m1, topo=topo)),
                     ("bf16 colmask 3 topo", dict(out16=o16, colmask=masks, topo=topo)),
                     ("bf16 colmask 3 topo clamp", dict(out16=o16, colmask=masks, topo=topo, clamp=(-1.0, 1.0))),
                     ("no output (K loop only)", dict())):
        print(f"tile {tile} {name}: {t(lambda: gemm(a, w, 'nt', tile=tile, **kw)):.1f} us", flush=True)
print(f"hipblaslt bf16: {t(lambda: torch.mm(a, w.t(), out=o16)):.1f} us")
print(f"memset bf16 out: {t(lambda: o16.zero_()):.1f} us")
