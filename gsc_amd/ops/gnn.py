"""Autograd wrappers around the native GATv2 embedder kernels: the fused per-graph MFMA kernels
(``csrc/ops/gnn_mf.hip`` for <= 32 nodes, ``gnn_mt.hip`` for 33..64 nodes, dispatched by ``gnn.hip``)
and, for every other shape (200-node topologies, wider embedders, other layer counts), the
layer-wise kernels (``gsc_amd/ops/gnn_lw.py``)."""
from __future__ import annotations

from typing import List

import torch

from gsc_amd.native import load as load_native


def _tables(graphs) -> dict:
    t = getattr(graphs, "_kernel_tables", None)
    if t is None:
        t = dict(src=graphs.src_i32.data_ptr(), dst=graphs.dst_i32.data_ptr(), in_ptr=graphs.in_ptr.data_ptr(),
                 in_msg=graphs.in_msg.data_ptr(), out_ptr=graphs.out_ptr.data_ptr(),
                 out_msg=graphs.out_msg.data_ptr(), deg=graphs.deg.data_ptr(), nnodes=graphs.n_nodes_i32.data_ptr(),
                 nmsgs=graphs.num_msgs.data_ptr(), M=int(graphs.M), NM=int(graphs.max_nodes),
                 in_src=graphs.in_src.data_ptr(), in_dst=graphs.in_dst.data_ptr(), out_q=graphs.out_q.data_ptr(),
                 out_dst=graphs.out_dst.data_ptr(), uniq=bool(graphs.unique_messages),
                 s_dst=graphs.s_dst.data_ptr(), s_src=graphs.s_src.data_ptr(), MP=int(graphs.mf_mp),
                 deg_order=graphs.deg_order.data_ptr())
        graphs._kernel_tables = t
    return t


def _layer_of(embedder) -> List[int]:
    seq = [0]
    if embedder.num_layers > 1:
        for _ in range(embedder.num_iter):
            seq.extend(range(1, embedder.num_layers))
    return seq


def _flat(params: List[torch.Tensor]) -> torch.Tensor:
    """Contiguous fp32 view of the embedder parameters (zero-copy when they already are one flat run)."""
    first = params[0]
    total = sum(p.numel() for p in params)
    base = first.data_ptr()
    contiguous = all(p.is_contiguous() for p in params)
    off = 0
    for p in params:
        if not contiguous or p.data_ptr() != base + off * 4 or p.dtype != torch.float32:
            return torch.cat([q.detach().reshape(-1).float() for q in params])
        off += p.numel()
    return first.detach().reshape(-1) if total == first.numel() else \
        torch.as_strided(first.detach(), (total,), (1,))


_PARTIALS = {}


class _GnnEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, topo, graphs, meta, *params):
        nat = load_native()
        B, P, Fin = x.shape
        H, layer_of, grad_mode = meta
        flat = _flat(list(params))
        x = x.contiguous().float()
        topo = topo.to(torch.int32).contiguous()
        emb = torch.empty(B, H, device=x.device, dtype=torch.float32)
        # grad-requiring forward: save the per-layer state for the backward (MFMA path) instead of
        # having it recompute the forward
        nbytes = nat.gnn_saved_bytes(_tables(graphs), P, Fin, H, layer_of) if grad_mode and any(ctx.needs_input_grad[4:]) \
            else 0
        blob = torch.empty(B * nbytes if B > 0 else 0, device=x.device, dtype=torch.uint8)
        if B > 0:
            nat.gnn_forward(_tables(graphs), flat.data_ptr(), x.data_ptr(), topo.data_ptr(), emb.data_ptr(), B, P, Fin,
                            H, layer_of, torch.cuda.current_stream(x.device).cuda_stream,
                            blob.data_ptr() if blob.numel() else 0)
        ctx.save_for_backward(x, topo, flat, blob)
        ctx.graphs, ctx.meta = graphs, meta
        ctx.shapes = [p.shape for p in params]
        return emb

    @staticmethod
    def backward(ctx, demb):
        nat = load_native()
        x, topo, flat, blob = ctx.saved_tensors
        H, layer_of, _ = ctx.meta
        B, P, Fin = x.shape
        grad = torch.empty_like(flat)
        rows = 1024
        stream = torch.cuda.current_stream(x.device)
        key = (x.device, flat.numel(), stream.cuda_stream)  # concurrent branches must not share partials
        partials = _PARTIALS.get(key)
        if partials is None:
            partials = _PARTIALS[key] = torch.empty(rows, flat.numel(), device=x.device, dtype=torch.float32)
        nat.gnn_backward(_tables(ctx.graphs), flat.data_ptr(), x.data_ptr(), topo.data_ptr(),
                         demb.contiguous().float().data_ptr(), partials.data_ptr(), rows, grad.data_ptr(), B, P, Fin,
                         H, layer_of, stream.cuda_stream, blob.data_ptr() if blob.numel() else 0)
        out, off = [], 0
        for s in ctx.shapes:
            n = 1
            for d in s:
                n *= d
            out.append(grad[off:off + n].view(s))
            off += n
        return (None, None, None, None, *out)


def gnn_fits(embedder, graphs, P: int, Fin: int) -> bool:
    """The fused MFMA kernels cover this shape (<= 64 nodes, H <= 32, F_in <= 16, encoder + one
    shared process block, unique messages; per-graph working set within one CU's LDS)."""
    key = ("_gnn_fits", embedder.hidden_dim, tuple(_layer_of(embedder)), P, Fin)
    cache = graphs.__dict__.setdefault("_fits_cache", {})
    if key not in cache:
        cache[key] = bool(load_native().gnn_fused_fits(int(graphs.M), int(graphs.max_nodes), int(P), int(Fin),
                                                       int(embedder.hidden_dim), _layer_of(embedder),
                                                       bool(graphs.unique_messages)))
    return cache[key]


def gnn_use_fused(embedder, graphs, P: int, Fin: int) -> bool:
    """Fused per-graph MFMA kernels, or the layer-wise kernels for every shape they do not cover."""
    return gnn_fits(embedder, graphs, P, Fin)


def gnn_embed(embedder, x: torch.Tensor, topo: torch.Tensor, graphs) -> torch.Tensor:
    params = embedder.flat_parameters()
    return _GnnEmbed.apply(x, topo, graphs, (embedder.hidden_dim, _layer_of(embedder), torch.is_grad_enabled()), *params)


_LW_CACHE = {}


def _lw(graphs, B: int, P: int, Fin: int, H: int, layer_of, dev, fresh: bool):
    from .gnn_lw import LayerwiseGAT
    if fresh:
        return LayerwiseGAT(_tables(graphs), B, P, Fin, H, layer_of, dev)
    key = (id(graphs), B, P, Fin, H, tuple(layer_of), str(dev))
    lw = _LW_CACHE.get(key)
    if lw is None:
        lw = _LW_CACHE[key] = LayerwiseGAT(_tables(graphs), B, P, Fin, H, layer_of, dev)
    return lw


class _GnnEmbedLW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, topo, graphs, meta, *params):
        H, layer_of, grad_mode = meta
        B, P, Fin = x.shape
        flat = _flat(list(params)).contiguous()
        x = x.contiguous().float()
        topo32 = topo.to(torch.int32).contiguous()
        need = grad_mode and any(ctx.needs_input_grad[4:])
        lw = _lw(graphs, B, P, Fin, H, layer_of, x.device, fresh=need)
        emb = torch.empty(B, H, device=x.device, dtype=torch.float32)
        lw.forward(flat, x, topo32, emb, save=need)
        ctx.lw, ctx.flat, ctx.shapes = lw, flat, [p.shape for p in params]
        ctx.keep = (x, topo32)  # the saved forward references them
        return emb

    @staticmethod
    def backward(ctx, demb):
        grad = torch.empty_like(ctx.flat)
        ctx.lw.backward(ctx.flat, demb.contiguous().float(), grad)
        out, off = [], 0
        for sh in ctx.shapes:
            n = 1
            for d in sh:
                n *= d
            out.append(grad[off:off + n].view(sh))
            off += n
        return (None, None, None, None, *out)


def gnn_embed_layerwise(embedder, x: torch.Tensor, topo: torch.Tensor, graphs) -> torch.Tensor:
    params = embedder.flat_parameters()
    return _GnnEmbedLW.apply(x, topo, graphs, (embedder.hidden_dim, _layer_of(embedder), torch.is_grad_enabled()),
                             *params)
