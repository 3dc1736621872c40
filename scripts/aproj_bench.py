"""Time the fused TD-target projection kernel (csrc/ops/actor_proj.hip) at a given shape.

``python scripts/aproj_bench.py [--M 25600 --K 256 --A 360000 --J 64 --T 3 --iters 10]`` prints ms per call
and the achieved bf16 TFLOP/s (2 M A (K + J) flops).  Default shape: BASELINE config 5 (syn200, 3 SFCs,
three topologies, 100 samples per env-step at 256 envs).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gsc_amd.native import load as load_native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=25600)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--A", type=int, default=360000)
    ap.add_argument("--J", type=int, default=64)
    ap.add_argument("--T", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--slab-mb", type=int, default=64, help="split-K slab bytes (bounds the split count)")
    a = ap.parse_args()
    nat = load_native()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    A8 = (a.A + 7) // 8 * 8
    h = (torch.randn(a.M, a.K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(a.A, a.K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(a.A, device=dev, generator=g) * 0.1
    mask = (torch.rand(a.T, a.A, device=dev, generator=g) > 0.3).float()
    topo = torch.randint(0, a.T, (a.M,), device=dev, generator=g, dtype=torch.int32)
    wa = torch.zeros(a.J, A8, device=dev, dtype=torch.bfloat16)
    wa[:, :a.A] = (torch.randn(a.J, a.A, device=dev, generator=g) * 0.01).to(torch.bfloat16)
    slabs = torch.empty(a.slab_mb << 18, device=dev)
    z = torch.empty(a.M, a.J, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def run():
        return nat.actor_proj(h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), bias.data_ptr(), mask.data_ptr(),
                              mask.stride(0), a.T, topo.data_ptr(), wa.data_ptr(), wa.stride(0), a.M, a.K, a.A, a.J,
                              -1.0, 1.0, slabs.data_ptr(), slabs.numel(), z.data_ptr(), z.stride(0), s)

    S = run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / a.iters * 1e3
    fl = 2.0 * a.M * a.A * (a.K + a.J)
    print(f"actor_proj M={a.M} K={a.K} A={a.A} J={a.J} T={a.T} splits={S}: {ms:.3f} ms/call  "
          f"{fl / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
