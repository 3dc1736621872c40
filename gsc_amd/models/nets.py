"""Actor and critic (reference: ``src/rlsp/agents/models.py:55-154``).

Actor (graph mode): ``emb = GNN(obs)``; ``MLP([emb | mask]) * mask`` with PyG ``MLP`` semantics
(ReLU between layers, plain last layer, no norm) and **no output squashing** (Q6).
Critic: ``MLP([GNN(obs) | mask | action]) -> Q``.

Flat mode (``graph_mode: False``, reference ``models.py:115-122, 151``): the reference sizes the
actor's first layer for ``obs + action`` inputs but feeds only the flattened observation (Q13, a
shape error at the first forward).  Here flat mode is the evident intent: actor
``MLP(flatten(obs)) -> action``, critic ``MLP([flatten(obs) | action]) -> Q`` (no embedder, no mask
inputs; the actor output is still multiplied by the topology's action mask so padded nodes
schedule nothing).

The action mask is a per-topology constant, so its contribution to the first layer,
``mask @ W1[:, H:H+A]^T``, is evaluated once per topology and added like a bias instead of
multiplying a ``[B, A]`` block of known zeros/ones (bit-for-bit the same function and the same
gradients — autograd sees the mask columns of ``W1`` through that per-topology product).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from gsc_amd.ops.linear import composed_projection, linear, shadow
from .gnn import GNNEmbedder
from .graphs import GraphSet


def select_rows(table: torch.Tensor, topo: torch.Tensor) -> torch.Tensor:
    """``table[topo]`` for a per-topology table ``[T, D]``.

    A single topology broadcasts (no [B, D] materialisation, and the backward is a plain column
    sum); several topologies use a one-hot GEMM, whose backward is again a GEMM instead of an
    atomic scatter-add of B rows into T rows."""
    if table.shape[0] == 1:
        return table
    onehot = F.one_hot(topo, table.shape[0]).to(table.dtype)
    return onehot @ table


class MaskedInputMLP(nn.Module):
    """PyG-style MLP whose input is ``[dense | mask(topology) | extra]``; mask block folded per topology."""

    def __init__(self, dense_dim: int, mask_dim: int, extra_dim: int, hidden: Sequence[int], out_dim: int):
        super().__init__()
        self.dense_dim, self.mask_dim, self.extra_dim = dense_dim, mask_dim, extra_dim  # mask_dim 0: no mask input
        dims = [dense_dim + mask_dim + extra_dim, *hidden, out_dim]
        self.layers = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(dims) - 1)])

    @property
    def first(self) -> nn.Linear:
        return self.layers[0]

    def first_layer(self, dense, topo, masks, extra=None):
        W = self.first.weight
        W16 = shadow(W)
        sl = lambda a, b: (W[:, a:b], W16[:, a:b] if W16 is not None else None)
        D, A = self.dense_dim, self.mask_dim
        w, w16 = sl(0, D)
        h = linear(dense, w, self.first.bias, w16=w16)
        if A > 0:
            w, w16 = sl(D, D + A)
            topo_bias = linear(masks, w, w16=w16)            # [T, h1]
            h = h + select_rows(topo_bias, topo)
        if extra is not None:
            w, w16 = sl(D + A, W.shape[1])
            h = h + linear(extra, w, w16=w16)
        return h

    def forward(self, dense, topo, masks, extra=None, out_mask=None, out_mask16=None):
        """``out_mask`` [out_dim]: multiply the output by a constant 0/1 vector, folded into the last
        layer's weight rows and bias (same values as masking the ``[B, out]`` output, no extra pass)."""
        h = self.first_layer(dense, topo, masks, extra)
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            if i == 0:
                continue
            h = F.relu(h)
            if i == last and out_mask is not None:
                h = linear(h, layer.weight, layer.bias, row_mask=out_mask, row_mask16=out_mask16)
            else:
                h = linear(h, layer.weight, layer.bias)
        if last == 0 and out_mask is not None:
            h = h * out_mask
        return h

    def hidden(self, dense, topo, masks, extra=None):
        """Input of the last layer (post-ReLU activation of the last hidden layer)."""
        h = self.first_layer(dense, topo, masks, extra)
        for layer in self.layers[1:-1]:
            h = linear(F.relu(h), layer.weight, layer.bias)
        return F.relu(h)

    def forward_full(self, x):
        """Unfolded reference: ``x`` is the explicit concatenation (used by tests)."""
        h = x
        for i, layer in enumerate(self.layers):
            h = layer(h if i == 0 else F.relu(h))
        return h


def _embedder(cfg: dict, in_dim: int) -> GNNEmbedder:
    return GNNEmbedder(input_dim=in_dim, hidden_dim=int(cfg["GNN_features"]), num_layers=int(cfg["GNN_num_layers"]),
                       aggr=cfg.get("GNN_aggr", "mean"), num_iter=int(cfg["GNN_num_iter"]))


def _flat_dim(cfg: dict, obs_dim: int, action_dim: int) -> int:
    """Flattened observation size in flat mode: n_pad x obs features (n_pad from the action size)."""
    P = int(cfg.get("max_nodes", 24))
    return P * obs_dim


class Actor(nn.Module):
    def __init__(self, cfg: dict, obs_dim: int, action_dim: int, low=0.0, high=1.0):
        super().__init__()
        self.graph_mode = bool(cfg.get("graph_mode", True))
        self.action_dim = action_dim
        if self.graph_mode:
            self.embedder = _embedder(cfg, obs_dim)
            H, mdim = self.embedder.hidden_dim, action_dim
        else:
            self.embedder = None
            H, mdim = _flat_dim(cfg, obs_dim, action_dim), 0
        self.mlp = MaskedInputMLP(H, mdim, 0, list(cfg["actor_hidden_layer_nodes"]), action_dim)
        self.low, self.high = float(low), float(high)
        # reference: no output squashing (Q6); new optional key ``actor_output_activation: sigmoid``
        # bounds the policy to the [0, 1] action box (keeps the critic from being queried far outside
        # the replayed actions, where its linear extrapolation drives the actor loss to -inf)
        act = cfg.get("actor_output_activation", "none") or "none"
        if act not in ("none", "sigmoid"):
            raise ValueError(f"actor_output_activation must be none|sigmoid, got {act}")
        self.squash = act == "sigmoid"

    def embed(self, x, topo, graphs: GraphSet):
        return self.embedder(x, topo, graphs) if self.graph_mode else x.reshape(x.shape[0], -1)

    def forward(self, x, topo, graphs: GraphSet, masks: torch.Tensor):
        emb = self.embed(x, topo, graphs)
        if self.squash:
            return torch.sigmoid(self.mlp(emb, topo, masks)) * select_rows(masks, topo)
        if masks.shape[0] == 1:  # one topology: fold the output mask into the last layer
            m16 = shadow(masks)
            return self.mlp(emb, topo, masks, out_mask=masks[0], out_mask16=m16[0] if m16 is not None else None)
        out = self.mlp(emb, topo, masks)
        return out * select_rows(masks, topo)

    def hidden(self, x, topo, graphs: GraphSet, masks: torch.Tensor):
        """Last hidden activation ``z`` with ``forward(x) = (z W^T + b) * mask`` (W, b = last layer)."""
        return self.mlp.hidden(self.embed(x, topo, graphs), topo, masks)

    def scale_action(self, a):
        return 2.0 * ((a - self.low) / (self.high - self.low)) - 1.0

    def unscale_action(self, a):
        return self.low + (0.5 * (a + 1.0) * (self.high - self.low))


class QNetwork(nn.Module):
    def __init__(self, cfg: dict, obs_dim: int, action_dim: int):
        super().__init__()
        self.graph_mode = bool(cfg.get("graph_mode", True))
        if self.graph_mode:
            self.embedder = _embedder(cfg, obs_dim)
            H, mdim = self.embedder.hidden_dim, action_dim
        else:
            self.embedder = None
            H, mdim = _flat_dim(cfg, obs_dim, action_dim), 0
        self.mlp = MaskedInputMLP(H, mdim, action_dim, list(cfg["critic_hidden_layer_nodes"]), 1)

    def embed(self, x, topo, graphs: GraphSet):
        return self.embedder(x, topo, graphs) if self.graph_mode else x.reshape(x.shape[0], -1)

    def forward(self, x, topo, graphs: GraphSet, masks: torch.Tensor, action: torch.Tensor):
        emb = self.embed(x, topo, graphs)
        return self.mlp(emb, topo, masks, action)


    def forward_on_actor(self, x, topo, graphs: GraphSet, masks: torch.Tensor, actor: "Actor", z: torch.Tensor):
        """``forward(x, ..., actor(x))`` for one topology without materialising the ``[B, A]`` action.

        With one topology the actor output is ``a = z W2m^T + b2m`` (``W2m``, ``b2m``: last layer with
        the constant mask folded in), so the critic's action projection re-associates:
        ``a Wa^T = z (Wa W2m)^T + Wa b2m``.  Same function (up to rounding order); the ``[B, A]``
        actor output and its two large GEMMs (plus their backward) are replaced by an ``[H1, A] x
        [A, h]`` product and a ``[B, h] x [h, H1]`` GEMM.  Gradients reach the actor through
        ``W2m``, ``b2m`` and ``z`` exactly as through ``a``."""
        assert masks.shape[0] == 1, "composed critic/actor path needs a single topology"
        mlp = self.mlp
        D, A = mlp.dense_dim, mlp.mask_dim
        W1 = mlp.first.weight
        Wa = W1[:, D + A:]                                   # [h1, A]
        W16 = shadow(W1)
        if W16 is not None:
            Wa._bf16 = W16[:, D + A:]
        last = actor.mlp.layers[-1]
        m16 = shadow(masks)
        Mc, cb = composed_projection(Wa, last.weight, last.bias, masks[0],
                                     m16[0] if m16 is not None else None)   # [h1, z], [h1]
        emb = self.embed(x, topo, graphs)
        h = mlp.first_layer(emb, topo, masks) + linear(z, Mc, cb)
        for layer in mlp.layers[1:]:
            h = linear(F.relu(h), layer.weight, layer.bias)
        return h


def count_params(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())
