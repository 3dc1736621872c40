"""Fused Adam + Polyak (csrc/ops/optim.hip) at the config-5 actor size: device step counter, target, bf16 shadows.

    python scripts/adam_bench.py [--n 92600000] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=92_600_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from gsc_amd.native import load
    nat = load()
    n = a.n
    p, g, m, v, t = (torch.randn(n, device="cuda") * 0.01 for _ in range(5))
    v.abs_()
    p16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    t16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    step = torch.ones(1, device="cuda", dtype=torch.int64)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        nat.adam_polyak(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), t.data_ptr(), n, 1e-4, 0.9, 0.999, 1e-8,
                        1, 0.001, 1.0, 0.0, st, step_ptr=step.data_ptr(), skip_ptr=0, p16=p16.data_ptr(),
                        t16=t16.data_ptr())
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    gb = n * 40 / 1e9
    print(f"adam_polyak n={n}: {us:.1f} us ({gb / us * 1e6:.0f} GB/s at 40 B/param)", flush=True)


if __name__ == "__main__":
    main()
