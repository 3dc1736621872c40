"""Flat parameter buffers + fused Adam/Polyak (``csrc/ops/optim.hip``).

``FlatParams`` re-points every parameter of a module at a slice of one contiguous fp32 buffer,
so a whole network is one tensor for the optimizer kernel, for the Polyak update and for the
single data-parallel all-reduce of its gradient.  Semantics match ``torch.optim.Adam`` defaults
(the reference optimizer, ``simple_ddpg.py:162-163``) followed by the Polyak soft update
(``simple_ddpg.py:229-234``).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

import torch
import torch.nn as nn


class FlatParams:
    def __init__(self, module: nn.Module, align: int = 4, matrix_align: int = 8, bucket_align: int = 0):
        """``bucket_align`` > 0 (sharded optimizer, :mod:`gsc_amd.parallel.zero`): the block after the
        embedder and the buffer end start on multiples of it, so both buckets split into equal shards."""
        self.module = module
        self.matrix_align = matrix_align
        named = list(module.named_parameters())
        self.params: List[nn.Parameter] = [p for _, p in named]
        self.names = [n for n, _ in named]
        total = 0
        self.offsets = []
        self.split = 0  # first element after the embedder block (0: no embedder / no bucket split)
        seen_emb = False
        for name, p in named:
            emb = name.startswith("embedder.")
            if bucket_align and seen_emb and not emb and not self.split:
                total = -(-total // bucket_align) * bucket_align
                self.split = total
            seen_emb |= emb
            # MLP weight matrices start on a 16-byte boundary of the bf16 shadow (16-byte staging loads
            # in the MFMA GEMMs); the GNN block stays packed (its kernels index it as one run)
            if p.dim() == 2 and not emb:
                total = -(-total // matrix_align) * matrix_align
            self.offsets.append(total)
            total += p.numel()
        self.numel = total
        dev = self.params[0].device
        if bucket_align:
            align = bucket_align
        pad = (-total) % align
        self.flat = torch.zeros(total + pad, device=dev, dtype=torch.float32)
        for p, o in zip(self.params, self.offsets):
            self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
            p.data = self.flat[o:o + p.numel()].view_as(p)
        self.grad = torch.zeros_like(self.flat)
        self.flat16 = None

    def enable_shadow(self) -> None:
        """Keep a bf16 copy of the parameters (``param._bf16`` views) for the bf16 GEMMs.

        The fused Adam/Polyak kernel refreshes it in the same pass that writes the fp32 values, with
        the same round-to-nearest-even cast autocast would apply — so forwards need no cast kernels
        and produce bit-identical results."""
        self.flat16 = self.flat.to(torch.bfloat16)
        for p, o in zip(self.params, self.offsets):
            p._bf16 = self.flat16[o:o + p.numel()].view_as(p)

    def refresh_shadow(self) -> None:
        if self.flat16 is not None:
            self.flat16.copy_(self.flat)

    def offset_of(self, param: torch.Tensor) -> int:
        for p, o in zip(self.params, self.offsets):
            if p is param:
                return o
        raise KeyError("parameter not managed by this FlatParams")

    def view(self) -> torch.Tensor:
        return self.flat[: self.numel]

    def grad_view(self) -> torch.Tensor:
        return self.grad[: self.numel]

    def set_grads(self, grads: Iterable[Optional[torch.Tensor]]) -> torch.Tensor:
        """Write per-parameter gradients (``None`` = zero) into the flat gradient buffer.

        Runs of gradients that are consecutive slices of one buffer laid out like the parameters
        (e.g. the fused GNN backward's single gradient vector) are copied with one copy."""
        grads = list(grads)
        n = len(self.params)
        i = 0
        while i < n:
            g, o = grads[i], self.offsets[i]
            if g is None:
                self.grad[o:o + self.params[i].numel()].zero_()
                i += 1
                continue
            j = i + 1
            if g.is_contiguous():
                es, sp = g.element_size(), g.untyped_storage().data_ptr()
                while (j < n and grads[j] is not None and grads[j].is_contiguous() and grads[j].dtype == g.dtype
                       and grads[j].untyped_storage().data_ptr() == sp
                       and grads[j].data_ptr() == g.data_ptr() + (self.offsets[j] - o) * es):
                    j += 1
            length = self.offsets[j - 1] + self.params[j - 1].numel() - o
            src = g.reshape(-1) if j == i + 1 else torch.as_strided(g, (length,), (1,), g.storage_offset())
            self.grad[o:o + length].copy_(src)
            i = j
        return self.grad

    def load_flat_(self, src: torch.Tensor) -> None:
        self.flat[: self.numel].copy_(src[: self.numel])
        self.refresh_shadow()

    # -- layout-independent form (checkpoints) -------------------------------------------------------
    # The flat layout depends on bucket_align (ZeRO on/off, world size), so checkpoints store every
    # parameter-shaped tensor (weights, Adam moments) *packed*: the parameters' elements back to back in
    # named_parameters() order, no alignment padding.  Loading re-packs into the current layout.
    def packed_numel(self) -> int:
        return sum(p.numel() for p in self.params)

    def pack(self, t: torch.Tensor) -> torch.Tensor:
        """Packed copy of a flat-layout tensor (this buffer's layout) — layout-free checkpoint form."""
        return torch.cat([t[o:o + p.numel()].reshape(-1) for p, o in zip(self.params, self.offsets)])

    def unpack(self, packed: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Flat-layout tensor (padding zero) from a packed one."""
        if packed.numel() != self.packed_numel():
            raise ValueError(f"packed tensor has {packed.numel()} elements, the network {self.packed_numel()}")
        out = torch.zeros_like(self.flat) if out is None else out
        k = 0
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            out[o:o + n].copy_(packed[k:k + n])
            k += n
        return out

    def legacy_offsets(self) -> List[int]:
        """Offsets of the unsharded layout (bucket_align 0): the layout of format-2 checkpoints."""
        total, out = 0, []
        for name, p in zip(self.names, self.params):
            if p.dim() == 2 and not name.startswith("embedder."):
                total = -(-total // self.matrix_align) * self.matrix_align
            out.append(total)
            total += p.numel()
        return out

    def pack_legacy(self, t: torch.Tensor, align: int = 4) -> torch.Tensor:
        """Packed form of a tensor stored in the unsharded layout (pre-packed checkpoints).  Only the unsharded
        lengths are accepted -- the parameter run itself or the padded flat buffer (Adam moments): a checkpoint
        written with a sharded (bucket-aligned) layout is longer and shifted and would load wrong weights."""
        offs = self.legacy_offsets()
        end = offs[-1] + self.params[-1].numel()
        if t.numel() not in (end, end + (-end) % align):
            raise ValueError(f"legacy (unpacked) checkpoint tensor has {t.numel()} elements; the unsharded layout of "
                             f"this network has {end} (padded {end + (-end) % align}) -- a sharded-layout checkpoint "
                             "cannot be read: re-save it with this build (packed layout)")
        return torch.cat([t[o:o + p.numel()].reshape(-1) for p, o in zip(self.params, offs)])


class FusedAdamPolyak:
    """Adam over a :class:`FlatParams` buffer with an optional fused Polyak update of a target buffer."""

    def __init__(self, flat: FlatParams, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 target: Optional[FlatParams] = None, tau: float = 0.0):
        self.fp = flat
        self.lr, self.betas, self.eps, self.wd = float(lr), betas, float(eps), float(weight_decay)
        self.target, self.tau = target, float(tau)
        self.m = torch.zeros_like(flat.flat)
        self.v = torch.zeros_like(flat.flat)
        # the step counter lives on the device so a captured HIP graph advances it on every replay
        self.step_t = torch.zeros((), dtype=torch.int64, device=flat.flat.device)
        self._host_step = 0
        # non-finite gradient guard: [flag, skipped-count, bad-wave events, events seen] (no per-step reset);
        # a flagged step leaves params/moments/target
        # untouched (device-side decision, no host sync, works inside captured HIP graphs)
        self.guard = torch.zeros(4, dtype=torch.int32, device=flat.flat.device)
        self.guard_enabled = os.environ.get("GSC_GRAD_GUARD", "1") != "0"
        self.zero = None  # ZeroShards: sharded optimizer state (enable_zero)

    # -- sharded optimizer (ZeRO-1, gsc_amd/parallel/zero.py) -----------------------------------------
    def enable_zero(self, shards) -> None:
        """Keep Adam moments for this rank's shards only; :meth:`reduce_grads` fills ``gshard`` and
        :meth:`step` updates the shard, all-gathers the parameters and refreshes targets + shadows."""
        dev = self.fp.flat.device
        self.zero = shards
        n = shards.local_numel
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.gshard = torch.zeros(n, device=dev)
        self.zflag = torch.zeros(4, dtype=torch.int32, device=dev)

    def reduce_grads(self, bucket: Optional[int] = None, async_op: bool = True):
        """Reduce-scatter the flat gradient's bucket(s) into ``gshard``; returns waitable handles."""
        from gsc_amd.parallel.zero import reduce_scatter_bucket
        z = self.zero
        out = []
        for b in ([bucket] if bucket is not None else range(len(z.buckets))):
            lo, hi = z.buckets[b]
            off = z.local_off[b]
            h = reduce_scatter_bucket(self.fp.grad, lo, hi, self.gshard[off:off + z.chunk(b)], z.world, z.rank,
                                      async_op=async_op)
            if h is not None:
                out.append(h)
        return out

    def _zero_state(self, t: torch.Tensor) -> torch.Tensor:
        """Full-length copy of a sharded state tensor (all-gathered; collective)."""
        from gsc_amd.parallel.zero import all_gather_bucket
        z = self.zero
        full = torch.zeros_like(self.fp.flat)
        for b in range(len(z.buckets)):
            lo, hi = z.shard(b)
            full[lo:hi].copy_(t[z.local_off[b]:z.local_off[b] + z.chunk(b)])
            all_gather_bucket(full, *z.buckets[b], z.world, z.rank)
        return full

    def _zero_load(self, t: torch.Tensor, full: torch.Tensor) -> None:
        z = self.zero
        for b in range(len(z.buckets)):
            lo, hi = z.shard(b)
            t[z.local_off[b]:z.local_off[b] + z.chunk(b)].copy_(full[lo:hi])

    @torch.no_grad()
    def _step_zero(self, grad_scale: float) -> None:
        from gsc_amd.parallel.zero import agree_any, all_gather_bucket
        z = self.zero
        p, t = self.fp.flat, (self.target.flat if self.target is not None else None)
        g = self.gshard
        if p.is_cuda:
            from gsc_amd.native import load
            nat = load()
            stream = torch.cuda.current_stream(p.device).cuda_stream
            skip = 0
            if self.guard_enabled:
                nat.grad_guard_local(g.data_ptr(), g.numel(), self.zflag.data_ptr(), stream)
                agree_any(self.zflag)      # one decision on every rank (the shards differ)
                nat.grad_guard_apply(self.zflag.data_ptr(), self.guard.data_ptr(), self.step_t.data_ptr(), stream)
                skip = self.guard.data_ptr()
            else:
                self.step_t.add_(1)
            for b in range(len(z.buckets)):
                lo, hi = z.shard(b)
                off = z.local_off[b]
                nat.adam_polyak(p[lo:].data_ptr(), g[off:].data_ptr(), self.m[off:].data_ptr(), self.v[off:].data_ptr(),
                                0, hi - lo, self.lr, self.betas[0], self.betas[1], self.eps, 1, 0.0, float(grad_scale),
                                self.wd, stream, step_ptr=self.step_t.data_ptr(), skip_ptr=skip)
            for b in range(len(z.buckets)):
                all_gather_bucket(p, *z.buckets[b], z.world, z.rank)
            f16 = self.fp.flat16
            t16 = getattr(self.target, "flat16", None) if t is not None else None
            nat.polyak_shadow(p.data_ptr(), t.data_ptr() if t is not None else 0, p.numel(),
                              self.tau if t is not None else 0.0, f16.data_ptr() if f16 is not None else 0,
                              t16.data_ptr() if t16 is not None else 0, skip, stream)
            return
        if self.guard_enabled:
            # one decision on every rank (the shards differ); with the guard off every rank steps and
            # all-gathers unconditionally, like the unsharded path
            bad = torch.tensor([0 if bool(torch.isfinite(g).all()) else 1], dtype=torch.int32)
            agree_any(bad)
            if int(bad[0]):
                self.guard[1] += 1
                return
        self._host_step += 1
        self.step_t.add_(1)
        for b in range(len(z.buckets)):
            lo, hi = z.shard(b)
            off, c = z.local_off[b], z.chunk(b)
            adam_polyak_reference(p[lo:hi], g[off:off + c] * grad_scale, self.m[off:off + c], self.v[off:off + c],
                                  None, self._host_step, self.lr, self.betas, self.eps, 0.0, self.wd)
        for b in range(len(z.buckets)):
            all_gather_bucket(p, *z.buckets[b], z.world, z.rank)
        if t is not None:
            t.copy_(self.tau * p + (1 - self.tau) * t)

    @property
    def skipped_steps(self) -> int:
        return int(self.guard[1].item())

    @property
    def step_count(self) -> int:
        return int(self.step_t.item()) if self.step_t.is_cuda else self._host_step

    def state_dict(self) -> dict:
        """Full-length moments (sharded: all-gathered -- a collective, every rank calls it)."""
        z = getattr(self, "zero", None) is not None
        m, v = (self._zero_state(self.m), self._zero_state(self.v)) if z else (self.m, self.v)
        return {"m": m, "v": v, "step": self.step_count, "lr": self.lr, "betas": self.betas, "eps": self.eps}

    def load_state_dict(self, sd: dict) -> None:
        if getattr(self, "zero", None) is not None:
            self._zero_load(self.m, sd["m"].to(self.m.device))
            self._zero_load(self.v, sd["v"].to(self.v.device))
        else:
            self.m.copy_(sd["m"])
            self.v.copy_(sd["v"])
        self._host_step = int(sd["step"])
        self.step_t.fill_(int(sd["step"]))

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0) -> None:
        if getattr(self, "zero", None) is not None:
            self._step_zero(grad_scale)
            return
        p, g = self.fp.flat, self.fp.grad
        t = self.target.flat if self.target is not None else None
        if p.is_cuda:
            from gsc_amd.native import load
            nat = load()
            stream = torch.cuda.current_stream(p.device).cuda_stream
            skip = 0
            if self.guard_enabled:
                assert self.guard.numel() >= 4 and self.guard.dtype == torch.int32
                # a skipped step does not advance Adam's bias-correction counter (done on the device)
                nat.grad_guard(g.data_ptr(), self.fp.numel, self.guard.data_ptr(), stream, self.step_t.data_ptr())
                skip = self.guard.data_ptr()
            else:
                self.step_t.add_(1)
            nat.adam_polyak(p.data_ptr(), g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                            t.data_ptr() if t is not None else 0, p.numel(), self.lr, self.betas[0],
                            self.betas[1], self.eps, 1, self.tau if t is not None else 0.0,
                            float(grad_scale), self.wd, stream, step_ptr=self.step_t.data_ptr(), skip_ptr=skip,
                            p16=self.fp.flat16.data_ptr() if self.fp.flat16 is not None else 0,
                            t16=(self.target.flat16.data_ptr()
                                 if t is not None and getattr(self.target, "flat16", None) is not None else 0))
            return
        if self.guard_enabled and not bool(torch.isfinite(g).all()):
            self.guard[1] += 1
            return
        self._host_step += 1
        self.step_t.add_(1)
        adam_polyak_reference(p, g * grad_scale, self.m, self.v, t, self._host_step, self.lr, self.betas, self.eps,
                              self.tau, self.wd)


@torch.no_grad()
def adam_polyak_reference(p, g, m, v, target, step, lr, betas, eps, tau, weight_decay=0.0):
    b1, b2 = betas
    if weight_decay:
        g = g + weight_decay * p
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2s = (1 - b2 ** step) ** 0.5
    denom = (v.sqrt() / bc2s).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bc1))
    if target is not None:
        target.copy_(tau * p + (1 - tau) * target)
