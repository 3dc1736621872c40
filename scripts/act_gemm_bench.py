"""The acting forward's output layer at config-5 shapes -- mu = mask[topo] * (h W^T + b), [E, 256] x [A, 256]^T with
E = 256 envs and A = 360,000 (fp32 out, per-topology column mask) -- for every GEMM-engine tile shape and K depth.

    python scripts/act_gemm_bench.py [--E 256] [--A 360000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--E", type=int, default=256)
    ap.add_argument("--A", type=int, default=360000)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from gsc_amd.ops.mlp import gemm
    E, A, K = a.E, a.A, a.K
    h = (torch.randn(E, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(A, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(A, device="cuda") * 0.1
    masks = (torch.rand(3, A, device="cuda") > 0.3).float()
    topo = torch.randint(0, 3, (E,), device="cuda", dtype=torch.int32)
    out = torch.empty(E, A, device="cuda")
    ref = None
    for tile in (2, 3, 1, 0):
        for bk in (32, 64):
            def run():
                gemm(h, w, "nt", out32=out, bias=b, colmask=masks, topo=topo, tile=tile, bk=bk)
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            err = float((out - ref).abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            gb = (A * K * 2 + E * A * 4) / 1e9
            print(f"tile {tile} bk {bk}: {us:.1f} us ({gb / us * 1e6:.0f} GB/s W read + out write; max |diff| vs tile 2 "
                  f"{err:.2e})", flush=True)


if __name__ == "__main__":
    main()
