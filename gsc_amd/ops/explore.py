"""Exploration noise + schedule post-processing (reference ``simple_ddpg.py:182-201, 338-395``).

Per env: ``a = unscale(scale(mu(s)) + N(rand_mu, rand_sigma))`` clipped to ``[0, 1]`` (warm-up:
``U[0,1) * mask``), then for every ``(src, sfc, sf)`` slice of ``n_pad`` destination weights,
twice: zero weights below the threshold and renormalise (all-zero -> uniform ``round(1/P, 10)``,
residual of the rounded sum added to the first element that can absorb it).

``explore_postprocess`` dispatches to the fused HIP kernels for CUDA tensors (lane-parallel per
slice: 32 lanes up to n_pad 32, a wave with up to 4 weights per lane up to n_pad 256; fp64
arithmetic like the reference's Python floats) and to the vectorised PyTorch reference below
otherwise.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

ACCURACY = math.sqrt(torch.finfo(torch.float64).eps)


def _round10(x: torch.Tensor) -> torch.Tensor:
    return torch.round(x * 1e10) / 1e10


def normalize_slices_reference(p: torch.Tensor, threshold: float = 0.1, passes: int = 2) -> torch.Tensor:
    """p [..., P] float64 -> thresholded, normalised weights (vectorised reference)."""
    p = p.to(torch.float64)
    P = p.shape[-1]
    for _ in range(passes):
        p = torch.where(p >= threshold, p, torch.zeros_like(p))
        s = p.sum(-1, keepdim=True)
        uni = torch.full_like(p, round(1.0 / P, 10))
        div = _round10(p / torch.where(s == 0, torch.ones_like(s), s))
        keep = (1 - s).abs() <= ACCURACY
        out = torch.where(s == 0, uni, torch.where(keep, p, div))
        resid = 1 - out.sum(-1, keepdim=True)
        # first index whose value can absorb the residual
        ok = (out + resid) >= 0
        first = torch.argmax(ok.to(torch.int8), dim=-1, keepdim=True)
        add = torch.zeros_like(out).scatter_(-1, first, resid)
        p = out + add
    return p


def explore_postprocess_reference(mu: torch.Tensor, mask: torch.Tensor, n_pad: int, warmup: bool,
                                  rand_mu: float, rand_sigma: float, generator: Optional[torch.Generator] = None,
                                  threshold: float = 0.1, passes: int = 2) -> torch.Tensor:
    E, A = mu.shape
    if warmup:
        a = torch.rand(E, A, generator=generator, device=mu.device, dtype=torch.float32) * mask
    else:
        noise = torch.randn(E, A, generator=generator, device=mu.device, dtype=torch.float32) * rand_sigma + rand_mu
        scaled = 2.0 * mu.float() - 1.0 + noise
        a = (0.5 * (scaled + 1.0)).clamp(0.0, 1.0)
    out = normalize_slices_reference(a.double().view(E, A // n_pad, n_pad), threshold, passes)
    return out.view(E, A).float()


_PBITS: dict = {}


def mask_bitsets(mask: torch.Tensor, n_pad: int) -> torch.Tensor:
    """[T, A] mask table -> [T, A / n_pad, 4] int64: bit d of word q of row r = (mask[t, r n_pad + 64 q + d] > 0), the
    simulator's destination bitset of a row whose weights are all positive (the exploration kernel's early-exit
    rows).  Cached per table (data pointer, version, shape; the entry keeps the table alive)."""
    T, A = mask.shape
    key = (mask.data_ptr(), mask._version, T, A, n_pad)
    hit = _PBITS.get(key)
    if hit is not None:
        return hit[1]
    R = A // n_pad
    m = torch.zeros(T, R, 256, dtype=torch.int64, device=mask.device)
    m[:, :, :n_pad] = (mask.view(T, R, n_pad) > 0).to(torch.int64)
    bits = (m.view(T, R, 4, 64) << torch.arange(64, device=mask.device, dtype=torch.int64)).sum(-1)  # distinct bits
    if len(_PBITS) > 8:
        _PBITS.clear()
    _PBITS[key] = (mask, bits.contiguous())  # the table itself is held: its address cannot be reused meanwhile
    return _PBITS[key][1]


def explore_postprocess(mu: torch.Tensor, mask: torch.Tensor, n_pad: int, warmup: bool, rand_mu: float,
                        rand_sigma: float, seed: int, step: int, threshold: float = 0.1, passes: int = 2,
                        out: Optional[torch.Tensor] = None, topo: Optional[torch.Tensor] = None,
                        pmask: Optional[tuple] = None) -> torch.Tensor:
    """mu [E, A] actor output -> post-processed actions [E, A] (float32).  ``mask``: [E, A] per-env
    masks, or with ``topo`` [E] the per-topology table [T, A] (row ``topo[e]`` masks env e).  ``pmask``
    (device, ``BatchedSimulator.pmask_target()``): also write the simulator's destination bitsets."""
    if mu.is_cuda:
        from gsc_amd.native import load
        nat = load()
        E, A = mu.shape
        mu = mu.contiguous().float()
        mask = mask.contiguous().float()
        if topo is not None:
            topo = topo.to(torch.int64).contiguous()
        else:
            assert mask.shape[0] == E
        if out is None:
            out = torch.empty(E, A, device=mu.device, dtype=torch.float32)
        pbits = 0
        if pmask is not None and topo is not None and n_pad > 128 and n_pad % 8 == 0:
            key = (mask.data_ptr(), mask._version, mask.shape[0], A, n_pad)
            if key in _PBITS or not torch.cuda.is_current_stream_capturing():
                pbits = mask_bitsets(mask, n_pad).data_ptr()
        nat.explore_postprocess(mu.data_ptr(), mask.data_ptr(), topo.data_ptr() if topo is not None else 0,
                                out.data_ptr(), E, A, n_pad, int(warmup), float(rand_mu), float(rand_sigma),
                                int(seed) & 0xffffffff, int(step), float(threshold), int(passes),
                                torch.cuda.current_stream(mu.device).cuda_stream, pmask,
                                **({"pbits": pbits} if pbits else {}))
        return out
    if topo is not None:
        mask = mask.index_select(0, topo.to(torch.int64))
    g = torch.Generator(device=mu.device)
    g.manual_seed((int(seed) * 1000003 + int(step)) & 0x7fffffffffffffff)
    return explore_postprocess_reference(mu, mask, n_pad, warmup, rand_mu, rand_sigma, g, threshold, passes)
