"""Tensor-level wrappers of the MFMA GEMM engine (``csrc/ops/mlp.hip``).

``gemm(a, b, layout, ...)`` computes ``alpha * op(a) @ op(b)`` with the fused epilogue:

* layout ``"nt"``  — ``a`` [M, K] (rows), ``b`` [N, K] (an ``nn.Linear`` weight): ``a @ b.T``
* layout ``"tn"``  — ``a`` [K, M], ``b`` [K, N]: ``a.T @ b`` (weight gradients, K = batch)
* layout ``"nn"``  — ``a`` [M, K], ``b`` [K, N]: ``a @ b`` (input gradients ``dY @ W``)

Operands may be strided row views (``ld`` = row stride, last dim contiguous), bf16 or fp32 (fp32 is
rounded to bf16 while staging).  The output goes to ``out16`` (bf16) and/or ``out32`` (fp32) row views.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from gsc_amd.native import load as load_native

LAYOUTS = {"nt": 0, "tn": 1, "nn": 2}
_DT = {torch.bfloat16: 0, torch.float32: 1}


def _ld(t: torch.Tensor) -> int:
    assert t.dim() == 2 and t.stride(1) == 1, "operands must be row-major 2-D views"
    return t.stride(0)


_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 64), 3: (64, 128)}


_TILE_POLICY = os.environ.get("GSC_GEMM_TILE", "small")


def pick_tile(M: int, N: int) -> int:
    """0: 128x128, 1: 128x64, 2: 64x64 output tiles (4 waves).  Default ("small"): 64x64 everywhere --
    measured on MI355X at the learner's shapes (B = 25,600), the extra blocks of the small tile hide
    latency better than the larger tiles' operand reuse helps ([B,256]x[256,1728]: 98.6 vs 119 / 135 us;
    [B,1728]x[1728,64]: 38 vs 50 us).  "large": the largest tile that still gives >= 256 blocks."""
    if _TILE_POLICY == "small":
        return 2
    if M <= 64 or N <= 64:
        return 2 if M <= 64 else 1
    for t in (0, 1, 2):
        bm, bn = _TILES[t]
        if -(-M // bm) * -(-N // bn) >= 256:
            return t
    return 2


def auto_splits(M: int, N: int, K: int, tile: int, cap: int) -> int:
    """Split-K count for long reductions (weight gradients, K = batch): ~512 blocks, >= 256 K per split,
    at most ``cap`` fp32 slab elements.  Products that still leave each block a K loop longer than 4,096
    (the critic's action projection and its weight gradient at large A: [B, A] x [A, 64] with a few
    hundred output blocks) split further, to <= 4,096 K per split."""
    if K < 1024:
        return 1
    bm, bn = _TILES[tile]
    blocks = -(-M // bm) * -(-N // bn)
    lim = cap // max(M * N, 1)
    s = max(1, min(512 // blocks, K // 256, 256, lim))
    if K // s > 4096 and blocks < 1024:
        s = max(s, min(-(-K // 4096), 256, lim))
    return max(1, s)


def gemm(a: torch.Tensor, b: torch.Tensor, layout: str = "nt", *, out16: Optional[torch.Tensor] = None,
         out32: Optional[torch.Tensor] = None, alpha: float = 1.0, bias: Optional[torch.Tensor] = None,
         rowtab: Optional[torch.Tensor] = None, topo: Optional[torch.Tensor] = None,
         colmask: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
         rowscale: Optional[torch.Tensor] = None, relu: bool = False, sigmoid: bool = False,
         dsig: Optional[torch.Tensor] = None, gmul: Optional[torch.Tensor] = None,
         clamp=None, accumulate: bool = False, splits: Optional[int] = 1, slabs: Optional[torch.Tensor] = None,
         aug_t: int = -1, aug_topo: Optional[torch.Tensor] = None, tile: Optional[int] = None,
         bk: Optional[int] = None, stream: Optional[int] = None, a_rows: Optional[torch.Tensor] = None,
         b_rows: Optional[torch.Tensor] = None) -> None:
    """See module docstring.  ``splits=None`` picks a split-K count (needs ``slabs``).  ``aug_t >= 0`` appends ``1 + aug_t`` virtual columns to ``b`` (layouts
    tn/nn): a ones column and the one-hot of ``aug_topo`` (the row topology of ``b``).  ``a_rows`` / ``b_rows``
    (int32): the operand's stored row r is its physical row ``rows[r]`` (a sampled batch read in place from the
    replay ring); the logical row count is ``rows.numel()``."""
    nat = load_native()
    lay = LAYOUTS[layout]
    ar = a_rows.numel() if a_rows is not None else a.shape[0]   # logical stored rows
    br = b_rows.numel() if b_rows is not None else b.shape[0]
    if lay == 0:
        M, K = ar, a.shape[1]
        N = br
        assert b.shape[1] == K
    elif lay == 1:
        K, M = ar, a.shape[1]
        N = b.shape[1]
        assert br == K
    else:
        M, K = ar, a.shape[1]
        N = b.shape[1]
        assert br == K
    ep = {"alpha": float(alpha)}
    for nm, r in (("a_rows", a_rows), ("b_rows", b_rows)):
        if r is not None:
            assert r.dtype == torch.int32 and r.is_contiguous() and r.device == a.device
            ep[nm] = r.data_ptr()
    if aug_t >= 0:
        assert lay in (1, 2) and aug_topo is not None
        ep.update(aug_n0=N, aug_t=int(aug_t), aug_topo=aug_topo.data_ptr())
        N = N + 1 + aug_t
    if bias is not None:
        ep["bias"] = bias.data_ptr()
    if rowtab is not None:
        ep.update(rowtab=rowtab.data_ptr(), ld_rowtab=_ld(rowtab))
    # one-row tables (a single topology): every row uses row 0, read once per column
    tabs = [t for t in (rowtab, colmask) if t is not None]
    if tabs and all(t.shape[0] == 1 for t in tabs):
        ep["single_topo"] = 1
    if topo is not None:
        assert topo.dtype == torch.int32
        ep["topo"] = topo.data_ptr()
    if colmask is not None:
        ep.update(colmask=colmask.data_ptr(), ld_colmask=_ld(colmask))
    if gate is not None:
        assert gate.dtype == torch.bfloat16
        ep.update(gate=gate.data_ptr(), ld_gate=_ld(gate))
    if rowscale is not None:
        assert rowscale.dtype == torch.float32 and rowscale.is_contiguous()
        ep["rowscale"] = rowscale.data_ptr()
    if relu:
        ep["relu"] = 1
    if sigmoid:  # a = sigmoid(.) (* colmask); dsig <- s (1 - s) (* colmask), the actor backward's gate
        ep["sigmoid"] = 1
        if dsig is not None:
            assert dsig.dtype == torch.bfloat16
            ep.update(dsig=dsig.data_ptr(), ld_dsig=_ld(dsig))
    if gmul is not None:  # elementwise factor (may alias out16: each element is read before it is written)
        assert gmul.dtype == torch.bfloat16
        ep.update(gmul=gmul.data_ptr(), ld_gmul=_ld(gmul))
    if clamp is not None:
        ep["clamp"] = (float(clamp[0]), float(clamp[1]))
    tile = pick_tile(M, N) if tile is None else int(tile)
    if bk is None:
        # K staged 32 deep per barrier.  BK = 64 is faster for two products in isolation (scripts/gemm_tune.py,
        # B = 25,600: [B,256]x[1728,256]^T 88.4 vs 93.0 us, [B,64]^T[B,1728] 40.0 vs 41.0 us) but lost in the
        # training step beside the concurrent kernels (bench.py 106.3k vs 106.9k env-steps/s)
        bk = 32
    if splits is None:
        splits = auto_splits(M, N, K, tile, slabs.numel()) if slabs is not None else 1
    eff = nat.gemm_splits(K, splits, bk) if splits > 1 else 1
    if accumulate and eff == 1:
        ep["accumulate"] = 1
    if eff > 1:
        assert (bias is None and rowtab is None and colmask is None and gate is None and rowscale is None and not relu
                and clamp is None and not sigmoid and gmul is None), "split-K supports alpha/accumulate only"
        assert slabs is not None and slabs.numel() >= eff * M * N, "split-K needs fp32 slabs"
        ep.update(c32=slabs.data_ptr(), ldc32=N, slab=M * N, splits=splits)
    else:
        if out32 is not None:
            assert out32.dtype == torch.float32
            ep.update(c32=out32.data_ptr(), ldc32=_ld(out32))
        if out16 is not None:
            assert out16.dtype == torch.bfloat16
            ep.update(c16=out16.data_ptr(), ldc16=_ld(out16))
    ep["tile"] = tile
    ep["bk"] = int(bk)
    s = torch.cuda.current_stream(a.device).cuda_stream if stream is None else stream
    nat.gemm(lay, M, N, K, a.data_ptr(), _ld(a), _DT[a.dtype], b.data_ptr(), _ld(b), _DT[b.dtype], ep, s)
    if eff > 1:
        assert out32 is not None, "split-K result goes to out32"
        nat.splitk_reduce(slabs.data_ptr(), M * N, eff, M, N, N, out32.data_ptr(), _ld(out32), float(alpha),
                          1 if accumulate else 0, s)
