"""Layer-wise GATv2 embedder on native kernels, for graphs too large for the fused per-graph
kernels (``gnn_fits`` false: e.g. the 200-node synthetic topologies of BASELINE config 5).

Per conv (``csrc/ops/gnn_lw.hip``): node linears ``x_l = h W_l^T + b_l``, ``x_r = h W_r^T + b_r``
(first conv: one pass over all ``B x P`` node rows -- the MFMA GEMM engine for inputs wider than 8
features; later convs: in the previous attention kernel's epilogue); attention + online segment softmax + mean aggregation (+ bias, ReLU) per
target node; mean pool per graph.  Backward: attention backward per target node (``d x_r`` gathered
per target, ``d x_l`` per source through the source-sorted CSR, with the input gradient
``dX W`` in the same gather), weight every parameter gradient of the conv (``dW = dX^T h``, bias / attention vectors) in one pass over its
rows with a deterministic two-phase reduction.  Same semantics as ``gatv2_dense_reference``
(reference ``src/rlsp/agents/models.py:10-53``).

A :class:`LayerwiseGAT` owns the workspaces of one batch size; ``forward`` keeps every conv's
output / ``x_l`` / ``x_r`` / attention weights (and a reference to its input) for the following
``backward``.
"""
from __future__ import annotations

from typing import List

import os

import torch

from gsc_amd.native import load as load_native
from .mlp import gemm


def _block_size(Fi: int, H: int) -> int:
    return 2 * H * Fi + 4 * H


def _block_offset(b: int, Fin: int, H: int) -> int:
    return 0 if b == 0 else _block_size(Fin, H) + (b - 1) * _block_size(H, H)


class LayerwiseGAT:
    def __init__(self, tables: dict, B: int, P: int, Fin: int, H: int, layer_of: List[int], device):
        self.nat = load_native()
        self.tables = tables
        self.B, self.P, self.Fin, self.H = int(B), int(P), int(Fin), int(H)
        self.layer_of = list(layer_of)
        self.L = len(self.layer_of)
        dev = torch.device(device)
        self.dev = dev
        R = self.B * self.P
        M = int(tables["M"])
        mk = lambda *s: torch.zeros(*s, device=dev, dtype=torch.float32)
        self.xl = [mk(R, H) for _ in range(self.L)]
        self.xr = [mk(R, H) for _ in range(self.L)]
        self.alpha = [mk(self.B, M) for _ in range(self.L)]
        self.hout = [mk(R, H) for _ in range(self.L)]
        self.x = None                      # layer-0 input of the saved forward
        # backward scratch
        self.dh = [mk(R, H), mk(R, H)]
        self.dxl, self.dxr, self.datt = mk(R, H), mk(R, H), mk(R, H)
        self.msg = mk(self.B * M, H)
        self.part = mk(1024 * max(H, 32))
        self.part_conv = mk(1024 * (2 * H * max(H, Fin) + 4 * H))   # per-block partials of lw_conv_grads
        self.vpart = mk(self.B, H)                                    # per-graph d att sums (staged backward)
        self.slabs = mk(max(4 << 20, 64 * H * max(H, Fin)))
        self.topo32 = None

    def _relu(self, l: int) -> bool:
        # ReLU after every conv but the last -- and after a single conv (GNNEmbedder.forward_reference)
        return l + 1 < self.L or self.L == 1

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _params(self, flat: torch.Tensor, blk: int):
        H, Fin = self.H, self.Fin
        Fi = Fin if blk == 0 else H
        o = _block_offset(blk, Fin, H)
        Wl = flat[o:o + H * Fi].view(H, Fi)
        o += H * Fi
        bl = flat[o:o + H]
        o += H
        Wr = flat[o:o + H * Fi].view(H, Fi)
        o += H * Fi
        br = flat[o:o + H]
        o += H
        att = flat[o:o + H]
        o += H
        bias = flat[o:o + H]
        return Fi, Wl, bl, Wr, br, att, bias

    def forward(self, flat: torch.Tensor, x: torch.Tensor, topo32: torch.Tensor, emb: torch.Tensor,
                save: bool = True) -> None:
        """flat: fp32 embedder parameters (module order); x [B, P, Fin] fp32; topo32 [B] int32; emb [B, H].
        save=False: no backward follows -- the staged kernels skip the per-conv output rows and alpha (the
        last conv's rows are read only as a ReLU gate, i.e. by a single-conv embedder)."""
        B, P, H = self.B, self.P, self.H
        assert x.shape == (B, P, self.Fin) and x.is_contiguous() and x.dtype == torch.float32
        assert topo32.dtype == torch.int32 and topo32.numel() == B
        nat, s, t = self.nat, self._stream(), self.tables
        self.x, self.topo32 = x, topo32
        h = x.view(B * P, self.Fin)
        for l, blk in enumerate(self.layer_of):
            Fi, Wl, bl, Wr, br, att, bias = self._params(flat, blk)
            first = ()
            if l == 0:   # later convs' node linears come from the previous attention kernel
                if Fi <= 8:   # computed inside the attention kernel (stored, coalesced, when a backward follows)
                    first = (h.data_ptr(), Fi, Wl.data_ptr(), bl.data_ptr(), Wr.data_ptr(), br.data_ptr(), int(save))
                else:
                    gemm(h, Wl, "nt", out32=self.xl[l], bias=bl)
                    gemm(h, Wr, "nt", out32=self.xr[l], bias=br)
            nxt = ()
            if l + 1 < self.L:
                _, Wl2, bl2, Wr2, br2, _, _ = self._params(flat, self.layer_of[l + 1])
                nxt = (Wl2.data_ptr(), bl2.data_ptr(), Wr2.data_ptr(), br2.data_ptr(), self.xl[l + 1].data_ptr(),
                       self.xr[l + 1].data_ptr())
            nat.lw_attn_fwd(t, topo32.data_ptr(), B, P, H, self.xl[l].data_ptr(), self.xr[l].data_ptr(),
                            att.data_ptr(), bias.data_ptr(), int(self._relu(l)), self.hout[l].data_ptr(),
                            self.alpha[l].data_ptr(), s, nxt, emb.data_ptr() if l + 1 == self.L else 0,
                            store=(1 if save and (l + 1 < self.L or self._relu(l)) else 0) | (2 if save else 0),
                            first=first)
            h = self.hout[l]   # the last conv also writes the mean pool into emb

    def backward(self, flat: torch.Tensor, demb: torch.Tensor, grad: torch.Tensor) -> None:
        """Gradients of the last ``forward`` into ``grad`` (fp32, module order; overwritten)."""
        B, P, H, R = self.B, self.P, self.H, self.B * self.P
        nat, s, t = self.nat, self._stream(), self.tables
        tp = self.topo32.data_ptr()
        cur, nxt = self.dh
        demb_c = demb.contiguous()   # the last conv's attention backward forms the pool backward itself
        seen = set()
        for l in range(self.L - 1, -1, -1):
            blk = self.layer_of[l]
            Fi, Wl, bl, Wr, br, att, bias = self._params(flat, blk)
            _, gWl, gbl, gWr, gbr, gatt, gbias = self._params(grad, blk)
            acc = blk in seen
            seen.add(blk)
            hin = self.x.view(R, self.Fin) if l == 0 else self.hout[l - 1]
            # attention backward + d x_l gather; l > 0: also the input gradient dxl W_l + dxr W_r into nxt
            # per-graph d att sums instead of [R, H] d att rows when the streamed gradient kernel applies
            stream_ok = H <= 32 and Fi <= 31 and os.environ.get("GSC_LW_STREAM_GRADS", "1") != "0"
            vsum = nat.lw_attn_bwd_gather(t, tp, B, P, H, cur.data_ptr(),
                                          self.hout[l].data_ptr() if self._relu(l) else 0,
                                          self.xl[l].data_ptr(), self.xr[l].data_ptr(), self.alpha[l].data_ptr(),
                                          att.data_ptr(), self.dxr.data_ptr(), self.msg.data_ptr(),
                                          self.datt.data_ptr(), self.dxl.data_ptr(), Wl.data_ptr() if l > 0 else 0,
                                          Wr.data_ptr() if l > 0 else 0, nxt.data_ptr() if l > 0 else 0, s,
                                          vpart=self.vpart.data_ptr() if stream_ok else 0,
                                          demb=demb_c.data_ptr() if l == self.L - 1 else 0)
            # dW_l | db_l | dW_r | db_r | d att | d bias in one pass (the block's layout in the flat gradient)
            assert gWl.data_ptr() == grad.data_ptr() + 4 * _block_offset(blk, self.Fin, H)
            if vsum:
                nat.lw_conv_grads_v(self.dxl.data_ptr(), self.dxr.data_ptr(), cur.data_ptr(), hin.data_ptr(), R, H, Fi,
                                    self.part_conv.data_ptr(), self.part_conv.numel(), gWl.data_ptr(), int(acc),
                                    self.vpart.data_ptr(), B, self.part.data_ptr(), s)
            else:
                nat.lw_conv_grads(self.dxl.data_ptr(), self.dxr.data_ptr(), self.datt.data_ptr(), cur.data_ptr(),
                                  hin.data_ptr(), R, H, Fi, self.part_conv.data_ptr(), self.part_conv.numel(),
                                  gWl.data_ptr(), int(acc), s)
            if l > 0:
                cur, nxt = nxt, cur
