"""GATv2 graph embedder (reference: ``src/rlsp/agents/models.py:10-53`` on PyG ``GATv2Conv``).

``GATv2Conv(in, out, aggr)`` with PyG defaults (1 head, concat, negative slope 0.2, self loops,
no dropout, ``share_weights=False``):

    x_l = x W_l^T + b_l,   x_r = x W_r^T + b_r
    e_ji = att . LeakyReLU_0.2(x_l[j] + x_r[i])           for every message j -> i (incl. self loop)
    a_ji = softmax_{j in N(i)} e_ji                        (segment softmax over the target node)
    out_i = AGGR_j(a_ji x_l[j]) + bias                     (aggr='mean' divides by the in-degree)

The embedder applies ``encoder -> ReLU`` then ``num_iter`` passes over the shared ``process``
convolutions (ReLU between, none after the last) and a mean pool over each graph's real nodes.

Two implementations with identical semantics:
* :func:`gatv2_dense_reference` — vectorised PyTorch (CPU path, autograd reference, tests);
* ``gsc_amd.ops.gnn`` — one fused HIP kernel per direction (whole embedder per graph in LDS),
  used automatically for CUDA tensors; graphs too large for LDS run the layer-wise native kernels
  (``gsc_amd/ops/gnn_lw.py``: MFMA GEMM node linears + per-node attention kernels).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .graphs import GraphSet

NEG_SLOPE = 0.2
# GSC_GNN_NATIVE=0: the PyTorch reference embedder on the GPU too (fp32 learning checks)
_NATIVE_GNN = os.environ.get("GSC_GNN_NATIVE", "1") != "0"
MAX_NATIVE_HIDDEN = 64  # widest GNN_features any native kernel family covers (csrc/ops/gnn_lw.hip)


def glorot_(t: torch.Tensor) -> torch.Tensor:
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        return t.uniform_(-a, a)


class GATv2Params(nn.Module):
    """Parameters of one ``GATv2Conv`` layer, initialised like PyG 2.3."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.in_ch, self.out_ch = in_ch, out_ch
        self.lin_l_weight = nn.Parameter(torch.empty(out_ch, in_ch))
        self.lin_l_bias = nn.Parameter(torch.empty(out_ch))
        self.lin_r_weight = nn.Parameter(torch.empty(out_ch, in_ch))
        self.lin_r_bias = nn.Parameter(torch.empty(out_ch))
        self.att = nn.Parameter(torch.empty(1, out_ch))
        self.bias = nn.Parameter(torch.empty(out_ch))
        self.reset_parameters()

    def reset_parameters(self):
        glorot_(self.lin_l_weight)
        glorot_(self.lin_r_weight)
        bound = 1.0 / math.sqrt(self.in_ch)
        with torch.no_grad():
            self.lin_l_bias.uniform_(-bound, bound)
            self.lin_r_bias.uniform_(-bound, bound)
            self.bias.zero_()
        glorot_(self.att)


def gatv2_dense_reference(x: torch.Tensor, src: torch.Tensor, dst: torch.Tensor, valid: torch.Tensor,
                          deg: torch.Tensor, p: GATv2Params) -> torch.Tensor:
    """x [B, N, Fin]; src/dst/valid [B, M]; deg [B, N] -> [B, N, H] (PyG GATv2Conv, aggr='mean')."""
    B, N, _ = x.shape
    xl = F.linear(x, p.lin_l_weight, p.lin_l_bias)
    xr = F.linear(x, p.lin_r_weight, p.lin_r_bias)
    H = xl.shape[-1]
    srcH = src.unsqueeze(-1).expand(-1, -1, H)
    dstH = dst.unsqueeze(-1).expand(-1, -1, H)
    xj = torch.gather(xl, 1, srcH)
    xi = torch.gather(xr, 1, dstH)
    e = (F.leaky_relu(xj + xi, NEG_SLOPE) * p.att.view(1, 1, H)).sum(-1)
    e = e.masked_fill(~valid, float("-inf"))
    with torch.no_grad():
        emax = torch.full((B, N), float("-inf"), device=x.device, dtype=e.dtype)
        emax = emax.scatter_reduce(1, dst, e, reduce="amax", include_self=True)
        emax = torch.where(torch.isfinite(emax), emax, torch.zeros_like(emax))
    ex = torch.exp(e - emax.gather(1, dst)) * valid
    den = torch.zeros((B, N), device=x.device, dtype=ex.dtype).scatter_add(1, dst, ex) + 1e-16
    alpha = ex / den.gather(1, dst)
    out = torch.zeros((B, N, H), device=x.device, dtype=xl.dtype).scatter_add(1, dstH, alpha.unsqueeze(-1) * xj)
    return out / deg.unsqueeze(-1) + p.bias


class GNNEmbedder(nn.Module):
    def __init__(self, input_dim: int, hidden_dim: int, num_layers: int, aggr: str = "mean", num_iter: int = 1,
                 dropout: float = 0.5):
        super().__init__()
        if aggr != "mean":
            raise NotImplementedError("GSC uses GNN_aggr: mean (the only aggregation implemented natively)")
        self.input_dim, self.hidden_dim = input_dim, hidden_dim
        self.num_layers, self.num_iter = num_layers, num_iter
        self.dropout = dropout  # stored but unused, as in the reference (Q21)
        self.encoder = GATv2Params(input_dim, hidden_dim)
        self.process = nn.ModuleList([GATv2Params(hidden_dim, hidden_dim) for _ in range(num_layers - 1)])

    def layer_sequence(self) -> List[GATv2Params]:
        seq = [self.encoder]
        if self.num_layers > 1:
            for _ in range(self.num_iter):
                seq.extend(self.process)
        return seq

    def flat_parameters(self) -> List[torch.Tensor]:
        return [t for m in [self.encoder, *self.process] for t in m.parameters()]

    def reset_parameters(self):
        self.encoder.reset_parameters()
        for p in self.process:
            p.reset_parameters()

    def forward(self, x: torch.Tensor, topo: torch.Tensor, graphs: GraphSet, use_native: Optional[bool] = None):
        """x [B, n_pad, F_in], topo [B] (topology index into ``graphs``) -> [B, hidden]."""
        if use_native is None:
            use_native = x.is_cuda and _NATIVE_GNN
        if use_native:
            if self.hidden_dim > MAX_NATIVE_HIDDEN:
                raise ValueError(f"GNN_features={self.hidden_dim}: the native GATv2 kernels cover at most "
                                 f"{MAX_NATIVE_HIDDEN} channels (MFMA <= 32, layer-wise <= 64); use a smaller "
                                 "GNN_features or GSC_GNN_NATIVE=0 (PyTorch reference embedder)")
            from gsc_amd.ops.gnn import gnn_embed, gnn_embed_layerwise, gnn_use_fused
            if gnn_use_fused(self, graphs, x.shape[1], x.shape[2]):
                return gnn_embed(self, x, topo, graphs)
            # shapes beyond the fused MFMA kernels (e.g. 200-node graphs): layer-wise native kernels
            return gnn_embed_layerwise(self, x, topo, graphs)
        return self.forward_reference(x, topo, graphs)

    def forward_reference(self, x, topo, graphs: GraphSet):
        src, dst, valid = graphs.src[topo], graphs.dst[topo], graphs.valid[topo]
        deg, nmask, nn_ = graphs.deg[topo], graphs.node_mask[topo], graphs.n_nodes[topo]
        seq = self.layer_sequence()
        h = x
        for i, p in enumerate(seq):
            h = gatv2_dense_reference(h, src, dst, valid, deg, p)
            if i < len(seq) - 1 or len(seq) == 1:
                h = F.relu(h)
        return (h * nmask.unsqueeze(-1)).sum(1) / nn_.unsqueeze(-1)
