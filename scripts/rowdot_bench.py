"""Bit-mask fold (csrc/ops/mlp.hip rowdot) at config-5 shapes: out[t][n] = sum_a mask_t[a] W[n][H + a], W the actor's
first layer (256 rows, H = 22 embedding columns before the A = 360,000-column mask block), T = 3 topologies.
GSC_ROWDOT_VEC=0 selects the 4-byte pair loop.

    python scripts/rowdot_bench.py [--N 256] [--A 360000] [--H 22]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--A", type=int, default=360000)
    ap.add_argument("--H", type=int, default=22)
    ap.add_argument("--T", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from gsc_amd.agents.native_update import mask_bits
    from gsc_amd.native import load
    nat = load()
    N, A, H, T = a.N, a.A, a.H, a.T
    W = (torch.randn(N, H + A, device="cuda") * 0.05).bfloat16()
    masks = (torch.rand(T, A, device="cuda") > 0.3).float()
    bits = mask_bits(masks)
    ws = torch.zeros(64 * T * N, device="cuda")
    out = torch.empty(T, N, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        nat.rowdot(masks.data_ptr(), masks.stride(0), T, W.data_ptr() + 2 * H, W.stride(0), N, A, out.data_ptr(),
                   out.stride(0), st, ws.data_ptr(), ws.numel(), bits.data_ptr(), bits.shape[1])
    run()
    torch.cuda.synchronize()
    ref = masks @ W[:, H:].float().t()
    err = float((out - ref).norm() / ref.norm())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(f"rowdot N={N} A={A} T={T} vec={os.environ.get('GSC_ROWDOT_VEC', '1')}: {us:.1f} us "
          f"({N * A * 2 / us / 1e3:.0f} GB/s of W; rel err vs fp32 {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
