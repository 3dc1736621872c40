"""Linear layer for the learner's bf16 GEMMs: bf16 parameter shadows + split-K weight gradients.

* **Shadows.**  Under autocast, ``F.linear`` casts the fp32 weight and bias to bf16 on every call
  (~70 small cast kernels per DDPG update).  Parameters managed by :class:`FlatParams` carry a
  ``_bf16`` view of a bf16 copy that the fused Adam/Polyak kernel rewrites in the same pass
  (identical rounding), so the forward uses it directly; the gradient still flows to the fp32
  parameter.
* **Split-K weight gradient.**  The learner's layers see 25,600-row batches with 22-1,728 features,
  so ``dW = g^T x`` has a small result and a 25,600-long reduction; hipBLASLt tiles only the small
  output (90-100 us for ``[64 x 1728]`` on MI355X vs an 18 us memory bound).  A batched GEMM over
  K-chunks plus an fp32 sum runs in 32-40 us (``scripts/gemm_bench.py``).
* ``row_mask`` multiplies output rows of W (and b) by a constant 0/1 vector (the actor's action
  mask), in both directions of autograd.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

MIN_ROWS = 8192  # split-K only pays off for long reductions


def shadow(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """bf16 shadow of a FlatParams-managed tensor (or of a constant tagged with ``_bf16``)."""
    return getattr(t, "_bf16", None) if t is not None else None


def _chunks(rows: int) -> int:
    if rows < MIN_ROWS:
        return 1
    for c in (16, 8, 4):
        if rows % c == 0 and rows // c >= 512:
            return c
    return 1


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, w16, b16, m16, dtype):
        xc = x if x.dtype == dtype else x.to(dtype)
        wc = w16 if w16 is not None else w.to(dtype)
        bc = None
        if b is not None:
            bc = b16 if b16 is not None else b.to(dtype)
        if m16 is not None:
            wc = wc * m16.unsqueeze(1)
            bc = bc * m16 if bc is not None else None
        out = F.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc, m16)
        ctx.has_b = b is not None
        ctx.w_dtype, ctx.x_dtype = w.dtype, x.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        xc, wc, m16 = ctx.saved_tensors
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
            if m16 is not None:
                gw = gw * m16.float().unsqueeze(1)
            gw = gw.to(ctx.w_dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = g.float().sum(0)
            if m16 is not None:
                gb = gb * m16.float()
            gb = gb.to(ctx.w_dtype)
        return gx, gw, gb, None, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None, w16: Optional[torch.Tensor] = None,
           b16: Optional[torch.Tensor] = None, row_mask: Optional[torch.Tensor] = None,
           row_mask16: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear(x, w * row_mask[:, None], b * row_mask)`` with shadows / split-K on the GPU under autocast."""
    if not (x.is_cuda and torch.is_autocast_enabled("cuda")):
        if row_mask is not None:
            w = w * row_mask.unsqueeze(1)
            b = b * row_mask if b is not None else None
        return F.linear(x, w, b)
    dtype = torch.get_autocast_dtype("cuda")
    w16 = w16 if w16 is not None else shadow(w)
    b16 = b16 if b16 is not None else shadow(b)
    m16 = None
    if row_mask is not None:
        m16 = row_mask16 if row_mask16 is not None else shadow(row_mask)
        m16 = m16 if m16 is not None else row_mask.to(dtype)
    with torch.autocast("cuda", enabled=False):
        if not torch.is_grad_enabled() or not (w.requires_grad or x.requires_grad or
                                               (b is not None and b.requires_grad)):
            xc = x if x.dtype == dtype else x.to(dtype)
            wc = w16 if w16 is not None else w.to(dtype)
            bc = (b16 if b16 is not None else b.to(dtype)) if b is not None else None
            if m16 is not None:
                wc = wc * m16.unsqueeze(1)
                bc = bc * m16 if bc is not None else None
            return F.linear(xc, wc, bc)
        return _Linear.apply(x, w, b, w16, b16, m16, dtype)


class _ComposedProjection(torch.autograd.Function):
    """``Mc = Wa (W2 * m[:, None])``, ``cb = Wa (b2 * m)`` in bf16 from shadows; gradients to W2 and b2
    only (the critic weights ``Wa`` are frozen while the actor loss is differentiated)."""

    @staticmethod
    def forward(ctx, w2, b2, w2_16, b2_16, m16, wa16):
        w2m = w2_16 * m16.unsqueeze(1)
        b2m = b2_16 * m16
        ctx.save_for_backward(wa16, m16)
        ctx.dtypes = (w2.dtype, b2.dtype)
        return wa16 @ w2m, wa16 @ b2m

    @staticmethod
    def backward(ctx, g_mc, g_cb):
        wa16, m16 = ctx.saved_tensors
        mf = m16.float()
        gw2 = (wa16.t() @ g_mc.to(wa16.dtype)).float() * mf.unsqueeze(1)
        gb2 = (wa16.t().float() @ g_cb.float()) * mf
        return gw2.to(ctx.dtypes[0]), gb2.to(ctx.dtypes[1]), None, None, None, None


def composed_projection(wa: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, m: torch.Tensor,
                        m16: Optional[torch.Tensor] = None):
    """``(Wa @ (W2 * m[:, None]), Wa @ (b2 * m))`` — the critic's action projection of the actor's
    last layer.  Uses bf16 shadows on the GPU under autocast when the critic is frozen."""
    wa16, w2_16, b2_16 = shadow(wa), shadow(w2), shadow(b2)
    if (torch.is_autocast_enabled("cuda") and w2.is_cuda and not wa.requires_grad and wa16 is not None
            and w2_16 is not None and b2_16 is not None):
        m16 = m16 if m16 is not None else shadow(m)
        m16 = m16 if m16 is not None else m.to(torch.bfloat16)
        with torch.autocast("cuda", enabled=False):
            return _ComposedProjection.apply(w2, b2, w2_16, b2_16, m16, wa16)
    w2m = w2 * m.unsqueeze(1)
    return wa @ w2m, wa @ (b2 * m)
