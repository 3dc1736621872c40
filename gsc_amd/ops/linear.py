"""Linear layer whose weight gradient uses a split-K batched GEMM.

The learner's layers see batches of 25,600 rows and 22-1,728 features, so every weight gradient
``dW = g^T x`` is a GEMM with a small ``[out, in]`` result and a 25,600-long reduction.  hipBLASLt
tiles those over the small output only (one wave of tiles, 90-100 us on MI355X for ``[64 x 1728]``
against an 18 us memory bound); splitting the reduction into C chunks as a batched GEMM
(``[C, out, K/C] x [C, K/C, in]``) plus an fp32 sum over C runs in 32-40 us
(``scripts/gemm_bench.py``).  Forward and input gradient are unchanged GEMMs; under autocast the
operands are bf16 exactly as ``F.linear`` would use them.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

MIN_ROWS = 8192  # below this the plain GEMM is as fast


def _chunks(rows: int) -> int:
    for c in (16, 8, 4):
        if rows % c == 0 and rows // c >= 512:
            return c
    return 1


class _SplitKLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dtype):
        xc = x.to(dtype) if dtype is not None else x
        wc = w.to(dtype) if dtype is not None else w
        out = F.linear(xc, wc, b.to(xc.dtype) if b is not None else None)
        ctx.save_for_backward(xc, wc)
        ctx.has_b = b is not None
        ctx.w_dtype, ctx.x_dtype = w.dtype, x.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        xc, wc = ctx.saved_tensors
        g = g.to(xc.dtype).contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.mm(g, wc).to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            rows = g.shape[0]
            c = _chunks(rows)
            x2 = xc.reshape(rows, -1)
            if c > 1:
                gw = torch.bmm(g.view(c, rows // c, -1).transpose(1, 2), x2.view(c, rows // c, -1)).float().sum(0)
            else:
                gw = torch.mm(g.t(), x2).float()
            gw = gw.to(ctx.w_dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = g.float().sum(0).to(ctx.w_dtype)
        return gx, gw, gb, None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear`` with a split-K weight gradient for large GPU batches (plain ``F.linear`` otherwise)."""
    if not x.is_cuda or x.dim() != 2 or x.shape[0] < MIN_ROWS or not torch.is_grad_enabled() \
            or not (w.requires_grad or x.requires_grad):
        return F.linear(x, w, b)
    dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else None
    with torch.autocast("cuda", enabled=False):
        return _SplitKLinear.apply(x, w, b, dtype)
