"""MFMA GEMM engine on the learner's big forward shape ([25600,256] x [256,1728]): cost of each
fused epilogue term (bias, topology column mask, clamp, bf16 vs fp32 out) and of the tile shape."""
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


B, A, H1 = 25600, 1728, 256
d = "cuda"
bf = torch.bfloat16
z = torch.randn(B, H1, device=d, dtype=bf)
w2 = torch.randn(A, H1, device=d, dtype=bf)
bias = torch.randn(A, device=d)
masks = (torch.rand(1, A, device=d) > 0.5).float()
topo = torch.zeros(B, dtype=torch.int32, device=d)
o16 = torch.empty(B, A, device=d, dtype=bf)
o32 = torch.empty(B, A, device=d)
flops = 2 * B * A * H1
for tile in (0, 1):
    for name, kw in [("plain out16", dict(out16=o16)), ("plain out32", dict(out32=o32)),
                     ("+bias", dict(out16=o16, bias=bias)),
                     ("+bias+colmask", dict(out16=o16, bias=bias, colmask=masks, topo=topo)),
                     ("+bias+colmask+clamp", dict(out16=o16, bias=bias, colmask=masks, topo=topo, clamp=(-1., 1.)))]:
        us = bench(lambda: gemm(z, w2, "nt", tile=tile, **kw))
        print(f"tile{tile} {name:24s} {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
us = bench(lambda: torch.mm(z, w2.t(), out=o16))
print(f"hipBLASLt torch.mm          {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s")
