"""One DDPG update on hand-written kernels only (GPU path of :class:`DDPGLearner`).

Reference: ``SimpleDDPG._update_critic / _update_actor / _update_target_networks``
(``src/rlsp/agents/simple_ddpg.py:204-234``) on the networks of ``src/rlsp/agents/models.py:55-154``.
Per update, on a replay batch (obs, topo, action, reward, next_obs, done):

    y   = r + (1 - d) gamma Q'(s', clamp(mu'(s'), -1, 1))
    Lq  = mean (Q(s, a) - y)^2              -> critic grads -> [all-reduce] -> Adam + Polyak (critic)
    La  = -mean Q_new(s, mu(s))             -> actor grads  -> [all-reduce] -> Adam + Polyak (actor)

Every product runs on the MFMA GEMM engine (``csrc/ops/mlp.hip``) with fused epilogues, the GATv2
embedders on the MFMA GNN kernels, the output layer + losses in one head kernel, the optimizer in the
fused Adam/Polyak kernel -- no autograd, no hipBLASLt, no PyTorch elementwise kernels; all buffers are
preallocated, so the whole update is captured into HIP graphs.  Manual backward per layer:

    first layer   h0 = relu(emb W_d^T + b + mask[topo] W_m^T (+ act W_a^T))   (mask block folded per topology)
                  dW_d | db | S_t = dh0^T [emb | 1 | onehot(topo)],  dW_m = sum_t S_t (x) mask_t,
                  dW_a = dh0^T act,  d emb = dh0 W_d
    hidden        h = relu(x W^T + b):  dW = dh^T x,  db = dh^T 1,  dx = (dh W) * (x > 0)
    actor output  a = (h W^T + b) * mask[topo]           (target: clamped to [-1, 1])

The actor loss goes through the critic's action projection.  With at least one actor hidden layer the
projection re-associates per topology t (``a W_a^T = h (W_a diag(m_t) W)^T + W_a (b * m_t)``), so no
``[B, A]`` actor output is materialised: with T topologies the rows are expanded into T blocks
(``hx[r] = onehot(topo[r]) (x) h[r]``) and the T products ``Mc_t = W_a diag(m_t) W`` run as one GEMM
over ``K = A`` -- T (critic width) x (actor width) x A MACs instead of B x A x (actor width) per
product.  With ``T * critic width > min(B, 1024)`` (or ``GSC_COMPOSE=0``) the ``[B, A]`` output and
its gradient are materialised -- both paths are the same function.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from gsc_amd.native import load as load_native
from gsc_amd.ops.gnn import _layer_of, _tables, gnn_use_fused
from gsc_amd.ops.mlp import auto_splits, gemm


def mask_bits(masks: torch.Tensor) -> Optional[torch.Tensor]:
    """Pack 0/1 action masks [T, A] into uint32 words (bit a % 32 of word a // 32, as int32) for the
    bit variant of the mask-fold kernel (``rowdot(..., xbits=)``); None when a mask is not exactly 0/1."""
    import numpy as np
    m = masks.detach().float().cpu()
    if not bool(((m == 0) | (m == 1)).all()):
        return None
    T, A = m.shape
    W = -(-A // 32)
    b = np.zeros((T, W * 32), np.uint8)
    b[:, :A] = m.numpy().astype(np.uint8)
    packed = np.packbits(b.reshape(T, W, 4, 8), axis=-1, bitorder="little").reshape(T, W * 4)
    return torch.from_numpy(packed.view(np.int32).copy()).to(masks.device)

BF16 = torch.bfloat16
F32 = torch.float32


def sparse_fwd_splits(B: int, R: int, max_splits: int, dev=None) -> int:
    """Row-block splits of ``sparse_fwd`` (256 samples x R / S row blocks per workgroup, one workgroup per CU):
    the S in 1..min(R, max_splits, 64) whose ceil(B / 256) S workgroups best fill whole rounds of the device's
    CUs (at least two rounds): the smallest S within 95 % of a whole number of rounds (fewer partial sums to
    reduce), else the best."""
    cus = 256
    if dev is not None and torch.cuda.is_available():
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
    tiles = -(-B // 256)
    best, best_eff = 1, -1.0
    for S in range(1, max(1, min(R, max_splits, 64)) + 1):
        wgs = tiles * S
        rounds = -(-wgs // cus)
        eff = wgs / (rounds * cus) if rounds >= 2 else wgs / (2 * cus)
        if eff >= 0.95:
            return S
        if eff > best_eff + 1e-9:
            best, best_eff = S, eff
    return best


class _Net:
    """Pointers/views of one Actor or QNetwork inside its FlatParams (fp32 master, bf16 shadow, grad)."""

    def __init__(self, module, flat, grad: bool, H: int, A: int, is_critic: bool):
        self.m, self.fp = module, flat
        self.layers = list(module.mlp.layers)
        self.H, self.A = H, A
        self.is_critic = is_critic

    def w16(self, i):
        return self.layers[i].weight._bf16

    def w32(self, i):
        return self.layers[i].weight

    def b32(self, i):
        return self.layers[i].bias

    def gw(self, i):
        fp, p = self.fp, self.layers[i].weight
        o = fp.offset_of(p)
        return fp.grad[o:o + p.numel()].view_as(p)

    def gb(self, i):
        fp, p = self.fp, self.layers[i].bias
        o = fp.offset_of(p)
        return fp.grad[o:o + p.numel()].view_as(p)

    @property
    def nh(self) -> int:  # hidden layers
        return len(self.layers) - 1

    def width(self, i) -> int:
        return self.layers[i].weight.shape[0]

    def emb_ptr(self) -> int:
        return self.fp.flat.data_ptr()  # the embedder block is the first run of the flat buffer


class NativeDDPGUpdate:
    def __init__(self, learner, batch_size: int):
        from gsc_amd.agents.ddpg import DDPGLearner  # noqa: F401  (type reference)
        L = learner
        self.L = L
        self.nat = load_native()
        dev = L.device
        self.dev = dev
        self.B = B = int(batch_size)
        self.H = H = L.actor.embedder.hidden_dim
        self.A = A = L.actor.action_dim
        self.masks = L.masks.float().contiguous()          # [T, A]
        self.mbits = mask_bits(self.masks)                 # packed 0/1 masks for the mask fold
        self.T = T = self.masks.shape[0]
        self.gamma = float(L.gamma)
        self.actor = _Net(L.actor, L.actor_flat, True, H, A, False)
        self.critic = _Net(L.critic, L.critic_flat, True, H, A, True)
        self.tactor = _Net(L.target_actor, L.target_actor_flat, False, H, A, False)
        self.tcritic = _Net(L.target_critic, L.target_critic_flat, False, H, A, True)
        # bounded actor (actor_output_activation: sigmoid): a = sigmoid(h W^T + b) * mask.  The critic's
        # action projection cannot be re-associated through the sigmoid, so the [B, A] actor output is
        # materialised; its GEMM epilogue also writes the gate s (1 - s) * mask into the action-gradient
        # buffer, which the backward's dL/da GEMM multiplies in place (no extra pass, no autograd)
        self.squash = bool(L.actor.squash)
        c1 = self.critic.width(0)
        self.compose = (os.environ.get("GSC_COMPOSE", "1") != "0" and self.actor.nh >= 1
                        and T * c1 <= min(B, 1024) and not self.squash)
        # TD target: target actor output layer + target critic action projection in one kernel
        # (csrc/ops/actor_proj.hip, no [B, A] action matrix)
        hl0 = self.actor.width(self.actor.nh - 1) if self.actor.nh else 0
        self.fuse_target = (os.environ.get("GSC_FUSE_TARGET", "1") != "0" and self.actor.nh >= 1 and T <= 4
                            and c1 <= 64 and hl0 in (64, 128, 256) and A >= 8  # actor_proj.hip: A >= 8
                            and not self.squash)
        # [*, A] bf16 operands get rows padded to 8 columns (zeros): 16-byte aligned rows, so the GEMM
        # engine stages them with vector loads also when A % 8 != 0 (50-node topologies: A = 22,500)
        self.A8 = A8 = -(-A // 8) * 8
        self.graphs = L.graphs
        self.tables = _tables(L.graphs)
        self.layer_of = _layer_of(L.actor.embedder)
        self.P = L.graphs.n_pad
        mk = lambda *s, dt=F32: torch.zeros(*s, device=dev, dtype=dt)
        # activations
        self.emb = {k: mk(B, H) for k in ("ta", "tc", "c", "c2", "a")}
        self.hid_a = [mk(B, self.actor.width(i), dt=BF16) for i in range(self.actor.nh)]
        self.hid_ta = [mk(B, self.actor.width(i), dt=BF16) for i in range(self.actor.nh)]
        self.hid_c = [mk(B, self.critic.width(i), dt=BF16) for i in range(self.critic.nh)]
        # target action / materialised actor output (neither exists with the fused target + composed loss)
        self.act_buf = mk(B, A, dt=BF16) if not (self.fuse_target and self.compose) else None
        cmax = max(self.critic.width(i) for i in range(self.critic.nh))
        amax = max([self.actor.width(i) for i in range(self.actor.nh)] + [1])
        wmax = max(cmax, amax)
        self.hacc = mk(B, cmax)
        self.y = mk(B)
        self.dh = [mk(B, wmax, dt=BF16), mk(B, wmax, dt=BF16)]
        self.dact = mk(B, A, dt=BF16) if not self.compose else None
        self.demb = mk(B, H)
        self.wa = {k: mk(c1, A8, dt=BF16) for k in ("c", "tc")}  # aligned critic action blocks
        # per-topology masked blocks W_a diag(m_t), stacked [T * c1, A] (composed actor loss)
        self.wam = mk(T * c1, A8, dt=BF16)[:, :A] if self.compose else None
        self.rowtab = {k: mk(T, wmax) for k in ("a", "ta", "c", "tc")}
        self.aug = mk(wmax, max(H + 1 + T, 1))
        hl = self.actor.width(self.actor.nh - 1) if self.actor.nh else 1
        self.mc32 = mk(T * c1, hl)                           # Mc_t = W_a diag(m_t) W, stacked over t
        self.mc16 = mk(T * c1, hl, dt=BF16)                  # same, bf16 (d hx = dh0x Mc)
        self.mccat = mk(c1, T * hl, dt=BF16)                 # [Mc_0 | .. | Mc_T-1] (forward, K = T hl)
        self.cb = mk(T, c1)                                  # W_a (b * m_t) per topology (row table)
        self.dmc = mk(T * c1, hl + 1)
        self.hx = mk(B, T * hl, dt=BF16) if T > 1 else None  # topology-expanded actor hidden / critic grads
        self.dh0x = mk(B, T * c1, dt=BF16) if T > 1 else None
        self.splits = None                                   # auto split-K for the batch reductions
        # output tiles of the products that stream the [B, A] action block / the A-long weights at large A
        # (scripts/gemm_tune.py syn200 at B = 25,600, profiles/gemm_tune_syn200.txt): the critic's action
        # projection 4.87 -> 3.44 ms with 128-row tiles and 64-deep K stages, its weight gradient 4.36 -> 3.91 ms
        # with 64-deep stages, Mc 245 -> 144 us with 64 x 128 tiles.  They pay from A ~ 16k on: syn50 (A = 22,500)
        # 19.88k -> 20.33k env-steps/s (profiles/large_a_tiles_syn50_ab.txt); Abilene (A = 1,728) keeps 64 x 64 x 32
        self.big_tiles = ({"act": {"tile": 1, "bk": 64}, "dw": {"tile": 2, "bk": 64}, "mc": {"tile": 3}}
                          if A >= int(os.environ.get("GSC_LARGE_A_MIN", "16384"))
                          and os.environ.get("GSC_LARGE_A_TILES", "1") != "0" else {})
        # split-K slabs (bound the split count): 64 MB, or 32 splits of the actor projection's [B, 64] partials
        self.slabs = mk(max(16 << 20, 32 * self.B * 64) if self.A >= 8192 else 16 << 20)
        self.head_blocks = max(64, min(256, -(-B // 64)))    # one block per CU (>= 16 rows per wave)
        cm = self.critic.width(self.critic.nh - 1)
        self.part = mk(self.head_blocks * (cm + 3))
        self.metrics = mk(4)                                 # qf1_loss, qf1_values, actor_loss, -
        # GNN saved state / backward partials
        nat = self.nat
        Fin = L.actor.embedder.input_dim
        self.Fin = Fin
        ne = sum(p.numel() for p in L.actor.embedder.flat_parameters())
        self.ne = ne
        # shapes beyond the fused MFMA kernels (e.g. 200-node graphs): layer-wise GNN kernels, one
        # workspace per saved forward ("a", "c") plus one for forwards without a backward
        self.layerwise = not gnn_use_fused(L.actor.embedder, L.graphs, self.P, Fin)
        if self.layerwise:
            from gsc_amd.ops.gnn_lw import LayerwiseGAT
            self.lwo = {k: LayerwiseGAT(self.tables, B, self.P, Fin, H, self.layer_of, dev) for k in ("a", "c", "-")}
            self.blob = {"a": None, "c": None}
        else:
            # the grad-requiring forwards save their per-layer images for the backward (measured on
            # MI355X, 256 Abilene envs: 101.9k vs 101.2k env-steps/s against recomputing them in LDS)
            sb = nat.gnn_saved_bytes(self.tables, self.P, Fin, H, self.layer_of)
            self.blob = {k: torch.empty(B * sb, device=dev, dtype=torch.uint8) for k in ("a", "c")}
        self.gnn_rows = 1024
        self.gnn_partials = torch.empty(self.gnn_rows, ne, device=dev, dtype=F32)
        self.gnn_grad = mk(ne)
        self.topo32 = torch.zeros(B, dtype=torch.int32, device=dev)
        # replayed actions read in place from the ring: ``b.actions`` is then the ring and these are the
        # sampled rows (DeviceReplay.sample(actions=False)); None: ``b.actions`` is the gathered [B, A] batch
        self.act_rows: Optional[torch.Tensor] = None
        # sparse replay rings (DeviceReplay(sparse_rows=R), csrc/ops/sparse_act.hip): set_sparse() binds the
        # record ring; the critic's action products then run on the row records instead of a [B, A] block
        self.sparse = None

    def set_sparse(self, ring: torch.Tensor, R: int, P: int) -> None:
        if self.critic.width(0) != 64:
            raise ValueError("sparse replayed actions need the critic's first layer width 64 (GSC_SPARSE_REPLAY=0)")
        if P > 238:
            raise ValueError("sparse replayed actions: at most 238 destinations per row (GSC_SPARSE_REPLAY=0)")
        self.sparse = (ring, int(R), int(P))
        self.sp_wsum = torch.empty(int(R) * 64, dtype=torch.int32, device=self.dev)  # per-block W_a column sums
        # row-block splits of the forward (one 138 KB-LDS workgroup per CU): the split count whose workgroup
        # total best fills whole dispatch rounds of the CUs, within the split-K slabs
        self.sp_splits = sparse_fwd_splits(self.B, int(R), self.slabs.numel() // (self.B * 64), self.dev)

    # ------------------------------------------------------------------------------------------
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _gnn_fwd(self, net: _Net, x: torch.Tensor, out: torch.Tensor, save: Optional[torch.Tensor],
                 key: str = "-") -> None:
        if self.layerwise:
            self.lwo[key].forward(net.fp.flat[:self.ne], x, self.topo32, out, save=key != "-")
            return
        self.nat.gnn_forward(self.tables, net.emb_ptr(), x.data_ptr(), self.topo32.data_ptr(), out.data_ptr(), self.B,
                             self.P, self.Fin, self.H, self.layer_of, self._stream(),
                             save.data_ptr() if save is not None else 0)

    def _gnn_fwd2(self, na: _Net, nb: _Net, x: torch.Tensor, out_a: torch.Tensor, out_b: torch.Tensor) -> None:
        """Two embedders on the same graphs (target actor + target critic on next_obs): one launch of the
        fused MFMA kernels (one topology / input load per graph); two layer-wise passes otherwise."""
        if self.layerwise:
            self._gnn_fwd(na, x, out_a, None)
            self._gnn_fwd(nb, x, out_b, None)
            return
        self.nat.gnn_forward2(self.tables, na.emb_ptr(), nb.emb_ptr(), x.data_ptr(), self.topo32.data_ptr(),
                              out_a.data_ptr(), out_b.data_ptr(), self.B, self.P, self.Fin, self.H, self.layer_of,
                              self._stream())

    def _gnn_bwd(self, net: _Net, x: torch.Tensor, demb: torch.Tensor, blob: torch.Tensor, key: str = "-") -> None:
        # the embedder gradient is the first run of the network's flat gradient buffer
        if self.layerwise:
            self.lwo[key].backward(net.fp.flat[:self.ne], demb, net.fp.grad[:self.ne])
            return
        self.nat.gnn_backward(self.tables, net.emb_ptr(), x.data_ptr(), self.topo32.data_ptr(), demb.data_ptr(),
                              self.gnn_partials.data_ptr(), self.gnn_rows, net.fp.grad.data_ptr(), self.B, self.P,
                              self.Fin, self.H, self.layer_of, self._stream(), blob.data_ptr() if blob is not None else 0)

    def _rowtab(self, net: _Net, key: str) -> torch.Tensor:
        """mask[t] @ W_m^T for every topology t: the folded mask block of the first layer [T, h0]."""
        h0 = net.width(0)
        out = self.rowtab[key][:, :h0]
        w = net.w16(0)
        mb = self.mbits
        self.nat.rowdot(self.masks.data_ptr(), self.masks.stride(0), self.T, w.data_ptr() + 2 * self.H, w.stride(0),
                        h0, self.A, out.data_ptr(), out.stride(0), self._stream(), self.slabs.data_ptr(),
                        self.slabs.numel(), mb.data_ptr() if mb is not None else 0,
                        mb.shape[1] if mb is not None else 0)
        return out

    def _wa(self, net: _Net, key: str, colmask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Aligned copy of the critic's action block W[:, H+A:] (optionally column-masked): the [c1, A]
        view of rows padded to A8 columns (the padding stays zero)."""
        w = net.w16(0)
        dst = self.wa[key]
        H, A = self.H, self.A
        self.nat.copy2d(w.data_ptr() + 2 * (H + A), w.stride(0), dst.data_ptr(), dst.stride(0), dst.shape[0], A,
                        colmask.data_ptr() if colmask is not None else 0, self._stream())
        return dst[:, :A]

    def _first(self, net: _Net, emb, rowtab, out16, extra=None, wa=None, extra_rowtab=None, acc_ready=False,
               extra_rows=None):
        """h0 = relu(emb W_d^T + b + rowtab[topo] (+ extra wa^T + extra_rowtab[topo])) -> out16.
        ``acc_ready``: ``hacc`` already holds the action projection (fused target path).  ``extra_rows``:
        row r of ``extra`` is its physical row extra_rows[r] (replay ring read in place)."""
        h0 = net.width(0)
        acc = acc_ready
        if extra is not None:
            if extra_rowtab is not None:
                gemm(extra, wa, "nt", out32=self.hacc[:, :h0], rowtab=extra_rowtab, topo=self.topo32)
            else:   # K = A: split-K when the [B, h0] output alone gives few workgroups (large A)
                gemm(extra, wa, "nt", out32=self.hacc[:, :h0], splits=None, slabs=self.slabs, a_rows=extra_rows,
                     **self.big_tiles.get("act", {}))
            acc = True
        gemm(emb, net.w16(0)[:, :self.H], "nt", out16=out16, bias=net.b32(0), rowtab=rowtab, topo=self.topo32,
             relu=True, accumulate=acc, out32=self.hacc[:, :h0] if acc else None)

    def _hidden_fwd(self, net: _Net, acts: List[torch.Tensor]) -> None:
        for i in range(1, net.nh):
            gemm(acts[i - 1], net.w16(i), "nt", out16=acts[i], bias=net.b32(i), relu=True)

    def _hidden_bwd(self, net: _Net, acts: List[torch.Tensor], dh: torch.Tensor, grads: bool) -> torch.Tensor:
        """Back through hidden layers nh-1 .. 1; ``dh`` = gradient at the last hidden activation's
        pre-ReLU (already gated).  Returns the gated gradient at layer 0's pre-activation."""
        cur = 0
        bufs = self.dh
        for i in range(net.nh - 1, 0, -1):
            wi, wo = net.width(i - 1), net.width(i)
            if grads:
                gemm(dh, acts[i - 1], "tn", out32=net.gw(i), splits=self.splits, slabs=self.slabs)
                gemm(dh, acts[i - 1][:, :0], "tn", out32=net.gb(i).view(-1, 1), aug_t=0, aug_topo=self.topo32)
            nxt = bufs[cur][:, :wi] if dh.data_ptr() != bufs[cur].data_ptr() else bufs[cur ^ 1][:, :wi]
            gemm(dh, net.w16(i), "nn", out16=nxt, gate=acts[i - 1])
            dh = nxt
        return dh

    def _first_bwd(self, net: _Net, emb, dh0, extra=None, extra_rows=None) -> None:
        """Gradients of the first layer (dense, bias, mask block, optional action block) + d emb."""
        H, A, T = self.H, self.A, self.T
        h0 = net.width(0)
        aug = self.aug[:h0, :H + 1 + T]
        gemm(dh0, emb, "tn", out32=aug, aug_t=T, aug_topo=self.topo32, splits=self.splits, slabs=self.slabs)
        gw = net.gw(0)
        self.nat.first_layer_grad(aug.data_ptr(), h0, H, T, A, self.masks.data_ptr(), self.masks.stride(0),
                                  gw.data_ptr(), gw.stride(0), net.gb(0).data_ptr(), self._stream())
        if extra is not None:
            gemm(dh0, extra, "tn", out32=gw[:, H + A:], splits=self.splits, slabs=self.slabs, b_rows=extra_rows,
                 **self.big_tiles.get("dw", {}))
        gemm(dh0, net.w16(0)[:, :H], "nn", out32=self.demb)

    def _critic_tail(self, net: _Net, acts, mode: int, dh_out: Optional[torch.Tensor], b) -> None:
        last = net.nh
        h = acts[last - 1]
        w = net.w32(last)
        self.nat.mlp_head(h.data_ptr(), h.stride(0), self.B, h.shape[1], mode, w.data_ptr(), net.b32(last).data_ptr(),
                          self.gamma, b.rewards.data_ptr(), b.dones.data_ptr(), self.y.data_ptr(),
                          dh_out.data_ptr() if dh_out is not None else 0, dh_out.stride(0) if dh_out is not None else 0,
                          self.part.data_ptr() if mode else 0, self.head_blocks, self._stream())

    def _head_reduce(self, net: _Net, C: int, mode: int) -> None:
        nw = self.head_blocks
        s = self._stream()
        part = self.part.data_ptr()
        if mode == 1:  # dW | db of the output layer (contiguous in the grad buffer); loss, q mean
            gw = net.gw(net.nh)
            assert net.gb(net.nh).data_ptr() == gw.data_ptr() + 4 * C
            self.nat.splitk_reduce(part, C + 3, nw, 1, C + 1, C + 3, gw.data_ptr(), C + 1, 1.0, 0, s)
            self.nat.splitk_reduce(part + 4 * (C + 1), C + 3, nw, 1, 2, C + 3, self.metrics.data_ptr(), 2,
                                   1.0 / self.B, 0, s)
        else:          # actor loss = -mean q
            self.nat.splitk_reduce(part + 4 * (C + 2), C + 3, nw, 1, 1, C + 3, self.metrics.data_ptr() + 8, 1,
                                   -1.0 / self.B, 0, s)

    # ------------------------------------------------------------------------------------------
    def prepare(self, b) -> None:
        """Batch-dependent inputs the kernels share (int32 topology ids)."""
        self.topo32.copy_(b.topo)

    def stage_critic(self, b) -> None:
        """TD target (target nets) + critic loss + all critic gradients into ``critic_flat.grad``."""
        H, A = self.H, self.A
        ta, tc, c = self.tactor, self.tcritic, self.critic
        # target actor and target critic embedders on s' (one launch)
        self._gnn_fwd2(ta, tc, b.next_obs, self.emb["ta"], self.emb["tc"])
        # target actor on s'
        self._first(ta, self.emb["ta"], self._rowtab(ta, "ta"), self.hid_ta[0])
        self._hidden_fwd(ta, self.hid_ta)
        last = ta.nh
        if self.fuse_target:
            # a' W_a'^T with a' = clamp(mask * (h W^T + b), -1, 1) tile by tile in LDS -> hacc
            h, w, wa, c1 = self.hid_ta[last - 1], ta.w16(last), self._wa(tc, "tc"), tc.width(0)
            self.nat.actor_proj(h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), ta.b32(last).data_ptr(),
                                self.masks.data_ptr(), self.masks.stride(0), self.T, self.topo32.data_ptr(),
                                wa.data_ptr(), wa.stride(0), self.B, h.shape[1], A, c1, -1.0, 1.0,
                                self.slabs.data_ptr(), self.slabs.numel(), self.hacc.data_ptr(), self.hacc.stride(0),
                                self._stream())
            self._first(tc, self.emb["tc"], self._rowtab(tc, "tc"), self.hid_c[0], acc_ready=True)
        else:
            gemm(self.hid_ta[last - 1], ta.w16(last), "nt", out16=self.act_buf, bias=ta.b32(last), colmask=self.masks,
                 topo=self.topo32, clamp=(-1.0, 1.0), sigmoid=self.squash)
            # target critic on (s', a')
            self._first(tc, self.emb["tc"], self._rowtab(tc, "tc"), self.hid_c[0], extra=self.act_buf,
                        wa=self._wa(tc, "tc"))
        self._hidden_fwd(tc, self.hid_c)
        self._critic_tail(tc, self.hid_c, 0, None, b)
        # critic on (s, a): loss + gradients
        self._gnn_fwd(c, b.obs, self.emb["c"], self.blob["c"], key="c")
        rows = self.act_rows      # the ring itself, addressed by the sampled rows (no [B, A] batch copy)
        if self.sparse is not None:
            self._sparse_first(c, rows)
            acts = None
        else:
            acts = b.actions[:, :A]   # replay rows are padded to 8 columns (16-byte aligned)
            self._first(c, self.emb["c"], self._rowtab(c, "c"), self.hid_c[0], extra=acts, wa=self._wa(c, "c"),
                        extra_rows=rows)
        self._hidden_fwd(c, self.hid_c)
        C = c.width(c.nh - 1)
        dh = self.dh[0][:, :C]
        self._critic_tail(c, self.hid_c, 1, dh, b)
        self._head_reduce(c, C, 1)
        dh0 = self._hidden_bwd(c, self.hid_c, dh, grads=True)
        self._first_bwd(c, self.emb["c"], dh0, extra=acts, extra_rows=rows)
        if self.sparse is not None:
            self._sparse_wgrad(c, dh0, rows)
        self._gnn_bwd(c, b.obs, self.demb, self.blob["c"], key="c")

    # -- sparse replayed actions (csrc/ops/sparse_act.hip) ----------------------------------------------------
    def _sparse_first(self, c: _Net, rows: torch.Tensor) -> None:
        """Critic first layer on replayed sparse actions: hacc = a W_a^T from the row records (row-block partial
        sums + split-K reduction), then + emb W_d^T + bias + mask block (the shared epilogue GEMM)."""
        ring, R, P = self.sparse
        H, A, c1 = self.H, self.A, c.width(0)
        wa, st, S = self._wa(c, "c"), self._stream(), self.sp_splits
        self.nat.sparse_fwd(ring.data_ptr(), rows.data_ptr(), self.B, R, P, wa.data_ptr(), wa.stride(0), c1,
                            self.sp_wsum.data_ptr(), self.slabs.data_ptr(), S, st)
        self.nat.splitk_reduce(self.slabs.data_ptr(), self.B * c1, S, self.B, c1, c1, self.hacc.data_ptr(),
                               self.hacc.stride(0), 1.0, 0, st)
        self._first(c, self.emb["c"], self._rowtab(c, "c"), self.hid_c[0], acc_ready=True)

    def _sparse_wgrad(self, c: _Net, dh0: torch.Tensor, rows: torch.Tensor) -> None:
        """dW_a = dh0^T a from the row records: one workgroup per row block writes its [c1, n_pad] gradient."""
        ring, R, P = self.sparse
        H, A, c1 = self.H, self.A, c.width(0)
        gw = c.gw(0)[:, H + A:]
        self.nat.sparse_wgrad(ring.data_ptr(), rows.data_ptr(), self.B, R, P, dh0.data_ptr(), dh0.stride(0), c1,
                              gw.data_ptr(), gw.stride(0), self._stream())

    def stage_actor_fwd(self, b) -> None:
        """Actor embedding + hidden layers on s (independent of the critic step: overlaps its all-reduce)."""
        a = self.actor
        self._gnn_fwd(a, b.obs, self.emb["a"], self.blob["a"], key="a")
        self._first(a, self.emb["a"], self._rowtab(a, "a"), self.hid_a[0])
        self._hidden_fwd(a, self.hid_a)

    def stage_actor_grad(self, b) -> None:
        """Actor loss through the (updated, frozen) critic -> actor gradients into ``actor_flat.grad``."""
        H, A = self.H, self.A
        a, c = self.actor, self.critic
        self._gnn_fwd(c, b.obs, self.emb["c2"], None)
        hl = self.hid_a[a.nh - 1]
        last = a.nh
        rt_c = self._rowtab(c, "c")
        T, c1, hw = self.T, c.width(0), hl.shape[1]
        st = self._stream()
        if self.compose:
            wam = self.wam                                            # W_a diag(m_t), t = 0 .. T-1
            w = c.w16(0)
            for t in range(T):
                self.nat.copy2d(w.data_ptr() + 2 * (H + A), w.stride(0), wam[t * c1].data_ptr(), wam.stride(0), c1, A,
                                self.masks[t].data_ptr(), st)
            ks = max(16, auto_splits(T * c1, hw, A, self.big_tiles.get("mc", {}).get("tile", 2), self.slabs.numel()))
            gemm(wam, a.w16(last), "nn", out32=self.mc32, slabs=self.slabs, splits=ks,   # Mc_t = W_a diag(m_t) W
                 **self.big_tiles.get("mc", {}))
            self.nat.cast2d(self.mc32.data_ptr(), hw, self.mc16.data_ptr(), hw, T * c1, hw, st)
            for t in range(T):                                        # [Mc_0 | .. ]: row j holds Mc_t[j] at t*hw
                self.nat.cast2d(self.mc32[t * c1].data_ptr(), hw, self.mccat.data_ptr() + 2 * t * hw,
                                self.mccat.stride(0), c1, hw, st)
            bl = a.b32(last)                                          # cb_t = W_a (b * m_t)
            self.nat.rowdot(bl.data_ptr(), bl.numel(), 1, wam.data_ptr(), wam.stride(0), T * c1, A,
                            self.cb.data_ptr(), T * c1, st, self.slabs.data_ptr(), self.slabs.numel())
            hx = hl
            if T > 1:
                hx = self.hx
                self.nat.topo_expand(hl.data_ptr(), hl.stride(0), hx.data_ptr(), hx.stride(0), self.B, hw, T,
                                     self.topo32.data_ptr(), st)
            self._first(c, self.emb["c2"], rt_c, self.hid_c[0], extra=hx, wa=self.mccat, extra_rowtab=self.cb)
        else:
            wa = self._wa(c, "c")
            # sigmoid actor: dact <- s (1 - s) * mask, consumed by the dL/da GEMM below
            gemm(hl, a.w16(last), "nt", out16=self.act_buf, bias=a.b32(last), colmask=self.masks, topo=self.topo32,
                 sigmoid=self.squash, dsig=self.dact if self.squash else None)
            self._first(c, self.emb["c2"], rt_c, self.hid_c[0], extra=self.act_buf, wa=wa)
        self._hidden_fwd(c, self.hid_c)
        C = c.width(c.nh - 1)
        dh = self.dh[0][:, :C]
        self._critic_tail(c, self.hid_c, 2, dh, b)
        self._head_reduce(c, C, 2)
        dh0 = self._hidden_bwd(c, self.hid_c, dh, grads=False)      # gated grad at the critic's layer-0 pre-act
        dz = self.dh[1][:, :hw] if dh0.data_ptr() != self.dh[1].data_ptr() else self.dh[0][:, :hw]
        if self.compose:
            # per topology t (rows of dh0x hold dh0 in block topo[r]):  dMc_t | dcb_t = dh0x_t^T [h | 1];
            # dW = sum_t diag(m_t) W_a^T dMc_t;  db = sum_t diag(m_t) W_a^T dcb_t;  dh = (dh0x Mc) * (h > 0)
            dh0x = dh0
            if T > 1:
                dh0x = self.dh0x
                self.nat.topo_expand(dh0.data_ptr(), dh0.stride(0), dh0x.data_ptr(), dh0x.stride(0), self.B, c1, T,
                                     self.topo32.data_ptr(), st)
            gemm(dh0x, hl, "tn", out32=self.dmc, aug_t=0, aug_topo=self.topo32, splits=self.splits, slabs=self.slabs)
            gemm(self.wam, self.dmc[:, :hw], "tn", out32=a.gw(last))
            gemm(self.wam, self.dmc[:, hw:hw + 1], "tn", out32=a.gb(last).view(-1, 1))
            gemm(dh0x, self.mc16, "nn", out16=dz, gate=hl)
        else:
            gemm(dh0, wa, "nn", out16=self.dact, colmask=self.masks, topo=self.topo32,   # dL/da (masked)
                 gmul=self.dact if self.squash else None)                             # (* sigmoid gate)
            gemm(self.dact, hl, "tn", out32=a.gw(last), splits=self.splits, slabs=self.slabs)
            gemm(self.dact, hl[:, :0], "tn", out32=a.gb(last).view(-1, 1), aug_t=0, aug_topo=self.topo32)
            gemm(self.dact, a.w16(last), "nn", out16=dz, gate=hl)
        dh0a = self._hidden_bwd(a, self.hid_a, dz, grads=True)
        self._first_bwd(a, self.emb["a"], dh0a)

    def stage_actor_gnn_bwd(self, b) -> None:
        """The actor embedder's backward: writes only the first ``ne`` entries of ``actor_flat.grad``
        (the MLP part written by :meth:`stage_actor_grad` can be all-reduced meanwhile)."""
        self._gnn_bwd(self.actor, b.obs, self.demb, self.blob["a"], key="a")

    def last_metrics(self) -> dict:
        m = self.metrics
        return {"qf1_loss": m[0], "qf1_values": m[1], "actor_loss": m[2]}


class NativeAct:
    """Acting forward ``mu(s)`` of the E environments on the native kernels (fp32 output): the
    actor's embedder, first layer (topology mask block folded), hidden layers and masked output
    layer -- the same products as the update's actor stages, without autograd or hipBLASLt.
    Reference: ``Actor.forward`` (``src/rlsp/agents/models.py:119-154``)."""

    def __init__(self, learner, E: int):
        L = learner
        self.L, self.nat, self.E = L, load_native(), int(E)
        dev = L.device
        self.H, self.A = L.actor.embedder.hidden_dim, L.actor.action_dim
        self.net = _Net(L.actor, L.actor_flat, False, self.H, self.A, False)
        self.masks = L.masks.float().contiguous()
        self.T = self.masks.shape[0]
        self.tables = _tables(L.graphs)
        self.layer_of = _layer_of(L.actor.embedder)
        self.P, self.Fin = L.graphs.n_pad, L.actor.embedder.input_dim
        n = self.net
        self.emb = torch.zeros(E, self.H, device=dev)
        self.hid = [torch.zeros(E, n.width(i), device=dev, dtype=BF16) for i in range(n.nh)]
        self.rowtab = torch.zeros(self.T, n.width(0), device=dev)
        self.rowdot_ws = torch.zeros(64 * self.T * n.width(0), device=dev)   # split-A partials of the fold
        self.mbits = mask_bits(self.masks)
        self.out = torch.zeros(E, self.A, device=dev)
        self.topo32 = torch.zeros(E, dtype=torch.int32, device=dev)
        self._topo_ref, self._topo_ver = None, -1
        self.rowtab_owned, self.rowtab_dirty = False, True
        self.lw = None
        if not gnn_use_fused(L.actor.embedder, L.graphs, self.P, self.Fin):
            from gsc_amd.ops.gnn_lw import LayerwiseGAT
            self.lw = LayerwiseGAT(self.tables, E, self.P, self.Fin, self.H, self.layer_of, dev)
            self.ne = sum(p.numel() for p in L.actor.embedder.flat_parameters())

    @staticmethod
    def supported(learner) -> bool:
        return bool(learner.native_ok and len(learner.actor.mlp.layers) >= 2)

    def refresh_rowtab(self) -> None:
        """mask[t] @ W_m^T of the first layer for every topology (current stream).  The learner calls it
        right after each actor optimizer step (inside the captured update), so the acting chain -- the
        simulator's critical path -- does not recompute it every step (``rowtab_owned``); weight writes
        outside the optimizer (checkpoint load, shadow refresh) mark it dirty."""
        n, s = self.net, torch.cuda.current_stream(self.L.device).cuda_stream
        w = n.w16(0)
        self.nat.rowdot(self.masks.data_ptr(), self.masks.stride(0), self.T, w.data_ptr() + 2 * self.H, w.stride(0),
                        n.width(0), self.A, self.rowtab.data_ptr(), self.rowtab.stride(0), s, self.rowdot_ws.data_ptr(),
                        self.rowdot_ws.numel(), self.mbits.data_ptr() if self.mbits is not None else 0,
                        self.mbits.shape[1] if self.mbits is not None else 0)
        self.rowtab_dirty = False

    def __call__(self, obs: torch.Tensor, topo: torch.Tensor) -> torch.Tensor:
        n, s = self.net, torch.cuda.current_stream(self.L.device).cuda_stream
        assert obs.shape[0] == self.E and obs.is_contiguous() and obs.dtype == F32
        # topology ids change at episode ends only: convert once per tensor (the reference held
        # keeps its storage from being reused by another tensor)
        if topo is not self._topo_ref or topo._version != self._topo_ver:
            self.topo32.copy_(topo)
            self._topo_ref, self._topo_ver = topo, topo._version
        if self.lw is not None:
            self.lw.forward(n.fp.flat[:self.ne], obs, self.topo32, self.emb, save=False)
        else:
            self.nat.gnn_forward(self.tables, n.emb_ptr(), obs.data_ptr(), self.topo32.data_ptr(), self.emb.data_ptr(),
                                 self.E, self.P, self.Fin, self.H, self.layer_of, s, 0)
        w = n.w16(0)
        if not self.rowtab_owned or self.rowtab_dirty:
            self.refresh_rowtab()
        gemm(self.emb, w[:, :self.H], "nt", out16=self.hid[0], bias=n.b32(0), rowtab=self.rowtab, topo=self.topo32,
             relu=True)
        for i in range(1, n.nh):
            gemm(self.hid[i - 1], n.w16(i), "nt", out16=self.hid[i], bias=n.b32(i), relu=True)
        gemm(self.hid[n.nh - 1], n.w16(n.nh), "nt", out32=self.out, bias=n.b32(n.nh), colmask=self.masks,
             topo=self.topo32, sigmoid=bool(self.L.actor.squash))
        return self.out
