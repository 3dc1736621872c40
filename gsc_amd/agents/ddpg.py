"""DDPG learner + batched device trainer.

Learner (reference ``SimpleDDPG._update_critic/_update_actor/_update_target_networks``,
``simple_ddpg.py:204-234``), per update on a replay batch:

    y  = r + (1 - d) * gamma * Q'(s', clamp(mu'(s'), -1, 1))            (Q5: clamp kept)
    Lq = mse(Q(s, a), y)                   -> Adam(critic)  (+ Polyak of the critic target)
    La = -mean(Q(s, mu(s)))                -> Adam(actor)   (+ Polyak of the actor target)

Each network lives in one flat fp32 buffer (:class:`FlatParams`), so an update is: fused GNN
kernels + MLP GEMMs (bf16 autocast, fp32 master weights) + one all-reduce per network (data
parallel) + one fused Adam/Polyak kernel per network.  The critic's parameters are frozen while
the actor loss is differentiated (the reference computes and later discards those gradients).

Trainer: E environments of the batched simulator step in lockstep; one iteration =
act (actor forward) -> exploration + post-processing kernel -> simulator kernel -> replay add
-> ``updates_per_step`` learner updates of ``batch_size`` samples.
"""
from __future__ import annotations

import collections
import copy
import ctypes
import math
import os
import time
import warnings
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from gsc_amd.envs.common import schedule_threshold
from gsc_amd.models import Actor, GraphSet, QNetwork
from gsc_amd.ops import FlatParams, FusedAdamPolyak, explore_postprocess
from gsc_amd.parallel.dist import DistInfo, allreduce_sum_, broadcast_tensors
from gsc_amd.sim.batched import BatchedSimulator
from gsc_amd.utils.tracing import trace_range
from .replay import Batch, DeviceReplay


_DIAG_NO_LEARN = os.environ.get("GSC_DIAG_NO_LEARN", "0") == "1"


class DDPGLearner:
    def __init__(self, cfg: dict, obs_dim: int, action_dim: int, graphs: GraphSet, C: int, F_: int, device,
                 dist_info: Optional[DistInfo] = None, amp_bf16: Optional[bool] = None, seed: int = 0,
                 zero: Optional[bool] = None):
        """``zero``: data parallel with sharded optimizer state (reduce-scatter -> Adam on 1/W -> all-gather,
        :mod:`gsc_amd.parallel.zero`); None = ``GSC_DP_ZERO=1``.  Off by default: the all-reduce path hides its
        collectives behind the actor forward / embedder backward, while the sharded step exposes the
        parameter all-gathers (docs/ARCHITECTURE.md, "Data parallelism": it trades ~2.7 ms of exposed
        all-gather for ~0.8 ms of optimizer time and 1/W of the moments at config-5 scale, 8 ranks)."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.graphs = graphs
        self.dist = dist_info or DistInfo()
        torch.manual_seed(seed)
        self.actor = Actor(cfg, obs_dim, action_dim).to(self.device)
        self.critic = QNetwork(cfg, obs_dim, action_dim).to(self.device)
        self.target_actor = copy.deepcopy(self.actor)
        self.target_critic = copy.deepcopy(self.critic)
        if zero is None:
            zero = os.environ.get("GSC_DP_ZERO", "0") == "1"
        self.zero = bool(zero and self.dist.enabled)
        # bf16 gradient all-reduce (half the bytes on xGMI; fp32 master weights / moments): opt-in
        self.grad_bf16 = self.dist.enabled and not self.zero and os.environ.get("GSC_DP_GRAD_BF16", "0") == "1"
        ba = 8 * self.dist.world_size if self.zero else 0   # equal shards per bucket
        self.actor_flat = FlatParams(self.actor, bucket_align=ba)
        self.critic_flat = FlatParams(self.critic, bucket_align=ba)
        self.target_actor_flat = FlatParams(self.target_actor, bucket_align=ba)
        self.target_critic_flat = FlatParams(self.target_critic, bucket_align=ba)
        for m in (self.target_actor, self.target_critic):
            for p in m.parameters():
                p.requires_grad_(False)
        # identical replicas on every rank (a learner built with world_size 1 stays process-local even
        # inside a process group)
        if self.dist.enabled:
            broadcast_tensors([self.actor_flat.flat, self.critic_flat.flat, self.target_actor_flat.flat,
                               self.target_critic_flat.flat])
        lr = float(cfg.get("learning_rate", 1e-3))
        tau = float(cfg.get("target_model_update", 1e-4))
        self.gamma = float(cfg.get("gamma", 0.99))
        self.critic_opt = FusedAdamPolyak(self.critic_flat, lr=lr, target=self.target_critic_flat, tau=tau)
        self.actor_opt = FusedAdamPolyak(self.actor_flat, lr=lr, target=self.target_actor_flat, tau=tau)
        if self.zero:
            from gsc_amd.parallel.zero import ZeroShards, bucket_bounds
            r, w = self.dist.rank, self.dist.world_size
            # actor: [embedder | MLP] buckets (the MLP bucket is reduced while the embedder backward runs);
            # critic: one bucket (all its gradients exist at once)
            self.actor_opt.enable_zero(ZeroShards(bucket_bounds(self.actor_flat.flat.numel(), self.actor_flat.split),
                                                  r, w))
            self.critic_opt.enable_zero(ZeroShards(bucket_bounds(self.critic_flat.flat.numel(), 0), r, w))
        self.masks = graphs.action_masks(C, F_)
        self.amp = (self.device.type == "cuda") if amp_bf16 is None else bool(amp_bf16)
        if self.amp and self.device.type == "cuda":
            # bf16 shadows of all four networks, refreshed by the fused Adam/Polyak kernels
            for fp in (self.actor_flat, self.critic_flat, self.target_actor_flat, self.target_critic_flat):
                fp.enable_shadow()
            self.masks._bf16 = self.masks.to(torch.bfloat16)
        self.updates = 0
        self.last: Dict[str, torch.Tensor] = {}
        self._graphs = None
        self._graph_warm = 0
        self._a = None
        # GSC_COMPOSE=0 forces the materialised critic(obs, actor(obs)) path (A/B checks)
        self.compose_actor_critic = os.environ.get("GSC_COMPOSE", "1") != "0"
        # GPU: the update runs on hand-written kernels only (native_update.py); GSC_NATIVE_LEARNER=0
        # selects the autograd + PyTorch path (the CPU path, and the reference for the GPU tests)
        self.native_ok = (self.device.type == "cuda" and self.amp and self.actor.graph_mode
                          and os.environ.get("GSC_NATIVE_LEARNER", "1") != "0")
        self._native = None
        self._topo_ready = False
        self._act_native = None

    def _autocast(self):
        if self.amp:
            # no cast cache: weights are re-read after every optimizer step, and HIP-graph capture
            # must not keep cached casts alive across replays
            return torch.autocast(device_type=self.device.type, dtype=torch.bfloat16, cache_enabled=False)
        return torch.autocast(device_type=self.device.type, enabled=False)

    def refresh_shadows(self) -> None:
        """Re-derive the bf16 shadows after parameters were written outside the optimizer."""
        for fp in (self.actor_flat, self.critic_flat, self.target_actor_flat, self.target_critic_flat):
            fp.refresh_shadow()
        if self._act_native is not None:
            self._act_native.rowtab_dirty = True

    @torch.no_grad()
    def act(self, obs: torch.Tensor, topo: torch.Tensor) -> torch.Tensor:
        """Greedy actor output (fp32).  GPU: native kernels (:class:`NativeAct`) when the batch is the
        trainer's acting batch; otherwise the module forward."""
        na = self._act_native
        if na is not None and obs.shape[0] == na.E and obs.is_contiguous():
            return na(obs, topo)
        with self._autocast():
            return self.actor(obs, topo, self.graphs, self.masks).float()

    def enable_native_act(self, E: int) -> None:
        from .native_update import NativeAct
        if NativeAct.supported(self):
            self._act_native = NativeAct(self, E)

    def _allreduce(self, flat: FlatParams, lo: int = 0, hi: Optional[int] = None):
        """Issue the sum-all-reduce of ``flat.grad[lo:hi]`` (fp32, or bf16 with ``GSC_DP_GRAD_BF16=1``)."""
        if not self.dist.enabled:
            return None
        from gsc_amd.parallel.dist import GradReduce
        sl = slice(lo, hi)
        staging = None
        if self.grad_bf16:
            if getattr(flat, "grad16", None) is None:
                flat.grad16 = torch.zeros_like(flat.grad, dtype=torch.bfloat16)
            staging = flat.grad16[sl]
        return GradReduce(flat.grad[sl], staging)

    # -- update stages of the autograd path (CPU; GPU reference with GSC_NATIVE_LEARNER=0) -------
    def _target(self, b: Batch) -> torch.Tensor:
        g, masks = self.graphs, self.masks
        with torch.no_grad(), self._autocast():
            # the clamped target action stays bf16: the target critic consumes it as a GEMM operand
            a2 = self.target_actor(b.next_obs, b.topo, g, masks).clamp(-1, 1)
            q2 = self.target_critic(b.next_obs, b.topo, g, masks, a2).float().view(-1)
            return b.rewards + (1 - b.dones) * self.gamma * q2

    def _stage_critic(self, b: Batch) -> None:
        """TD target + critic loss -> critic gradients in ``critic_flat.grad``."""
        g, masks = self.graphs, self.masks
        y = self._target(b)
        with self._autocast():
            q = self.critic(b.obs, b.topo, g, masks, b.actions[:, :self.actor.action_dim]).float().view(-1)
            lq = F.mse_loss(q, y)
        grads = torch.autograd.grad(lq, self.critic_flat.params)
        self.critic_flat.set_grads(grads)
        self._lq, self._qv = lq.detach(), q.detach().mean()

    def _composed(self) -> bool:
        # one topology and at least one actor hidden layer: critic(obs, actor(obs)) re-associated
        return (self.compose_actor_critic and self.masks.shape[0] == 1 and len(self.actor.mlp.layers) > 1
                and not self.actor.squash and self.actor.graph_mode)

    def _stage_actor_fwd(self, b: Batch) -> None:
        with self._autocast():
            if self._composed():
                self._a = self.actor.hidden(b.obs, b.topo, self.graphs, self.masks)
            else:
                self._a = self.actor(b.obs, b.topo, self.graphs, self.masks)

    def _stage_actor_grad(self, b: Batch, inv_world: float) -> None:
        """Critic Adam/Polyak, then the actor loss through the frozen (updated) critic -> actor gradients."""
        self.critic_opt.step(grad_scale=inv_world)
        for p in self.critic_flat.params:
            p.requires_grad_(False)
        with self._autocast():
            if self._composed():
                q = self.critic.forward_on_actor(b.obs, b.topo, self.graphs, self.masks, self.actor, self._a)
            else:
                q = self.critic(b.obs, b.topo, self.graphs, self.masks, self._a)
            la = -q.float().mean()
        grads = torch.autograd.grad(la, self.actor_flat.params)
        for p in self.critic_flat.params:
            p.requires_grad_(True)
        self.actor_flat.set_grads(grads)
        self._la = la.detach()
        self._a = None

    def _stage_actor_opt(self, inv_world: float) -> None:
        self.actor_opt.step(grad_scale=inv_world)

    def native_update(self, batch_size: int):
        if self._native is None or self._native.B != batch_size:
            from .native_update import NativeDDPGUpdate
            self._native = NativeDDPGUpdate(self, batch_size)
        return self._native

    def topo32_buffer(self, batch_size: int) -> Optional[torch.Tensor]:
        """The int32 topology-id buffer the native update reads (a replay sampler can gather into it
        directly, see ``update_graphed(topo_ready=True)``), or None off the native path."""
        return self.native_update(batch_size).topo32 if self.native_ok else None

    def update(self, b: Batch) -> None:
        """One DDPG update, eager.

        Data parallel: the critic-gradient all-reduce is issued as soon as the critic gradients exist
        and runs on the communicator's stream while the actor's embedding + hidden layers (which do
        not read critic weights) run on the compute stream; the critic step waits for it.  The actor's
        MLP gradients are all-reduced while the actor embedder's backward runs; only the embedder's
        (small) gradient all-reduce is exposed before the actor step."""
        stages, split = self._stages(b, 1.0 / self.dist.world_size)
        self._run_stages([lambda f=f: f() for f in stages], split)
        self.updates += 1
        self.last = self._metrics_now()

    def _run_stages(self, run, split: int) -> None:
        """``run``: five callables (critic grads | actor fwd | critic step + actor MLP grads | actor
        embedder bwd | actor step) with the gradient all-reduces issued between them."""
        r1, r2, r3, r3b, r4 = run
        if self.zero:  # reduce-scatters instead of all-reduces (the optimizer steps all-gather the params)
            r1()
            hs = self.critic_opt.reduce_grads()
            r2()
            for h in hs:
                h.wait()
            r3()
            two = len(self.actor_opt.zero.buckets) == 2
            hs = self.actor_opt.reduce_grads(bucket=1) if (split and two) else []
            r3b()
            hs += self.actor_opt.reduce_grads(bucket=0) if (split and two) else self.actor_opt.reduce_grads()
            for h in hs:
                h.wait()
            r4()
            return
        r1()
        h_c = self._allreduce(self.critic_flat)
        r2()
        if h_c is not None:
            h_c.wait()
        r3()
        h_am = self._allreduce(self.actor_flat, split, None)
        r3b()
        h_ag = self._allreduce(self.actor_flat, 0, split) if split > 0 else None
        for h in (h_am, h_ag):
            if h is not None:
                h.wait()
        r4()

    # -- HIP-graph replay ----------------------------------------------------------------------
    def _stages(self, b: Batch, inv_world: float):
        """The update as five stages: critic gradients | actor forward | critic step + actor MLP
        gradients | actor embedder backward | actor step, and the split index of the actor's flat
        gradient (embedder first: ``grad[:split]`` is written by stage 4 only).  The critic all-reduce
        runs concurrently with stage 2, the actor MLP all-reduce with stage 4."""
        if self.native_ok:
            nu = self.native_update(b.obs.shape[0])

            topo_ready = self._topo_ready

            def s1():
                if not topo_ready:   # else the replay sampler gathered the int32 ids itself
                    nu.prepare(b)
                nu.stage_critic(b)

            def s3():
                self.critic_opt.step(grad_scale=inv_world)
                nu.stage_actor_grad(b)

            def s4():
                self.actor_opt.step(grad_scale=inv_world)
                self._after_actor_step()

            return [s1, lambda: nu.stage_actor_fwd(b), s3, lambda: nu.stage_actor_gnn_bwd(b), s4], nu.ne

        def s4_autograd():
            self._stage_actor_opt(inv_world)
            self._after_actor_step()

        return [lambda: self._stage_critic(b), lambda: self._stage_actor_fwd(b),
                lambda: self._stage_actor_grad(b, inv_world), lambda: None, s4_autograd], 0

    def _after_actor_step(self) -> None:
        # the acting forward's per-topology mask fold follows the new actor weights (see NativeAct)
        na = self._act_native
        if na is not None:
            na.refresh_rowtab()
            na.rowtab_owned = True

    def _metrics_now(self) -> Dict[str, torch.Tensor]:
        if self.native_ok and self._native is not None:
            return self._native.last_metrics()
        return {"qf1_loss": self._lq, "actor_loss": self._la, "qf1_values": self._qv}

    def update_graphed(self, b: Batch, warmup: int = 2, pre=None, topo_ready: bool = False) -> None:
        """Same update, replayed from captured HIP graphs (``b`` must be the same static buffers on
        every call).  One graph for the whole update; data parallel (native learner): the gradient
        all-reduces are captured in it too (``GSC_DP_GRAPH=0``, or a failed capture: five graphs with
        the all-reduces issued eagerly between them).  Either way the critic all-reduce overlaps the
        actor forward, the actor-MLP all-reduce the actor embedder backward.  The first ``warmup`` calls run eagerly
        (they are real updates) on a side stream.  ``pre`` (e.g. the replay sampler filling ``b``)
        runs first and is captured with the update; ``topo_ready``: ``pre`` also fills
        :meth:`topo32_buffer`."""
        inv_world = 1.0 / self.dist.world_size
        self._topo_ready = bool(topo_ready and pre is not None)
        if self.zero:
            # the sharded optimizer step issues collectives between its kernels: eager (an update at the
            # scale that enables it runs for milliseconds; launch overhead is noise there)
            if pre is not None:
                pre()
            self.update(b)
            return
        if self._graphs is None:
            if self._graph_warm < warmup:
                s = torch.cuda.Stream(self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    if pre is not None:
                        pre()
                    self.update(b)
                torch.cuda.current_stream(self.device).wait_stream(s)
                self._graph_warm += 1
                return
            self._capture(b, inv_world, pre)
        if len(self._graphs) == 1:
            self._graphs[0].replay()
        else:
            self._run_stages([g.replay if g is not None else (lambda: None) for g in self._graphs], self._split)
        self.updates += 1
        self.last = self._metrics_now()

    def _capture(self, b: Batch, inv_world: float, pre=None) -> None:
        # thread-local capture: the RCCL watchdog thread keeps querying its events while we capture
        pool = torch.cuda.graph_pool_handle()
        stages, self._split = self._stages(b, inv_world)
        if pre is not None:
            s1 = stages[0]
            stages[0] = lambda: (pre(), s1())
        if (self.dist.enabled and self.native_ok and self.dist.backend == "nccl"
                and os.environ.get("GSC_DP_GRAPH", "1") != "0"):
            # data parallel over RCCL, one graph: the gradient all-reduces are captured with the stages (collectives
            # in a HIP graph: the communicator's stream forks off the learner stream and joins back, so the
            # critic all-reduce still overlaps the actor forward and the actor-MLP one the embedder backward).
            # Measured on a world-size-1 RCCL group, 256-env headline: 120.9k env-steps/s vs 121.2k process-local;
            # five graphs with eager collectives between them ran at 62-67k (profiles/dp_graph_ab.txt).
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                    self._run_stages(stages, self._split)
                self._graphs = [g]
                return
            except RuntimeError as e:  # a runtime / RCCL build without collective capture: per-stage graphs
                warnings.warn(f"capturing the DP update with its collectives failed ({e}); replaying per-stage "
                              "graphs with eager collectives")
                torch.cuda.synchronize(self.device)
        graphs = []
        # one process: one graph; data parallel: one graph per stage (collectives between them, eager);
        # a stage that launches nothing (autograd path's embedder stage) gets no graph
        groups = [stages] if not self.dist.enabled else [[f] for f in stages]
        for k, grp in enumerate(groups):
            if self.dist.enabled and not self.native_ok and k == 3:
                graphs.append(None)
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                for fn in grp:
                    fn()
            graphs.append(g)
        self._graphs = graphs
        # capture recorded but did not execute the update: the caller's replay performs it

    # checkpointing --------------------------------------------------------------------------
    # Parameters and Adam moments are stored packed (per parameter, no alignment padding): the flat layout
    # depends on the ZeRO bucket alignment (world size), the packed form does not, so a checkpoint resumes
    # under any rank count with or without the sharded optimizer.  ZeRO: state_dict is a collective.
    _NETS = (("actor", "actor_flat"), ("critic", "critic_flat"), ("target_actor", "target_actor_flat"),
             ("target_critic", "target_critic_flat"))

    def state_dict(self) -> dict:
        sd = {"layout": "packed", "updates": self.updates}
        for key, attr in self._NETS:
            fp = getattr(self, attr)
            sd[key] = fp.pack(fp.flat.detach()).clone()
        for key, opt in (("actor_opt", self.actor_opt), ("critic_opt", self.critic_opt)):
            o = opt.state_dict()
            o["m"], o["v"] = opt.fp.pack(o["m"]).clone(), opt.fp.pack(o["v"]).clone()
            sd[key] = o
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Every rank validates every tensor's length before any collective runs (a mismatch raises on all
        ranks alike instead of leaving some of them blocked in the ZeRO moment scatter)."""
        packed = sd.get("layout") == "packed"
        tens = {}
        for key, attr in self._NETS:
            fp = getattr(self, attr)
            t = sd[key].to(self.device).reshape(-1)
            tens[key] = fp.unpack(t if packed else fp.pack_legacy(t))
        opts = {}
        for key, opt in (("actor_opt", self.actor_opt), ("critic_opt", self.critic_opt)):
            o = {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in sd[key].items()}
            for mk in ("m", "v"):
                o[mk] = opt.fp.unpack(o[mk] if packed else opt.fp.pack_legacy(o[mk]))
            opts[key] = o
        for key, attr in self._NETS:
            getattr(self, attr).load_flat_(tens[key])
        self.actor_opt.load_state_dict(opts["actor_opt"])
        self.critic_opt.load_state_dict(opts["critic_opt"])
        self.updates = int(sd.get("updates", 0))
        if self._act_native is not None:  # weights written outside the optimizer
            self._act_native.rowtab_dirty = True


@dataclass
class TrainerConfig:
    num_envs: int = 256
    batch_size: Optional[int] = None        # default: 100 * num_envs (reference: 100 samples per env step)
    updates_per_step: int = 1
    learning_starts: Optional[int] = None   # iterations; default: nb_steps_warmup_critic
    replay_capacity: Optional[int] = None   # default: mem_limit * num_envs (capped)
    replay_cap_max: int = 2_000_000
    replay_bytes_max: Optional[float] = None  # default: 60 % (dense) / 65 % (sparse rows) of this process's
                                            # share of the device memory (_replay_hbm); 4 GB on CPU
    handoff_timeout_s: float = 10.0         # act <-> simulator sequence-word wait limit (then the run fails)
    seed: int = 0
    check_every: int = 50
    overlap_sim: bool = True                # run the simulator kernel on its own stream, concurrent with updates
    sim_cus: int = -1                       # >0: simulator stream owns this many CUs (contiguous CU-mask bits,
                                            # = sim_cus/8 per XCD), the learner the rest; 0: shared CUs;
                                            # -1: auto (enough CUs for one round of env waves, <= half the GPU)
    cuda_graphs: bool = True                # replay the DDPG update from captured HIP graphs (GPU only)
    amp_bf16: Optional[bool] = None         # None: bf16 GEMM operands on the GPU, fp32 on CPU; False: fp32
                                            # autograd learner everywhere (learning checks)
    lazy_handoff: bool = False              # overlap mode: hand work between the caller's stream and the
                                            # trainer's streams only at the trainer's read/write points
                                            # (metrics/flush/state_dict/load_state_dict/reseed), not around every
                                            # step -- saves two cross-stream event hops per step; the caller must
                                            # not touch trainer tensors between steps without those (or a device sync)
    act_on_sim_stream: bool = os.environ.get("GSC_ACT_ON_SIM", "1") == "1"  # overlap mode: the actor forward + exploration of step t+1 run on the
                                            # simulator's stream right behind step t's simulator kernel (after the
                                            # learner's update t), so the act -> simulate chain has no cross-stream
                                            # hop; the learner waits for the act (it reads the actor weights)


def replay_plan(cap: int, n_pad: int, n_obs: int, action_dim: int, action_bytes: int, hbm: float, eligible: bool,
                mode: str = "auto"):
    """(sparse, bytes per transition, byte budget) of the replay ring for ``cap`` requested transitions.

    Dense rows take ``action_bytes`` per action entry within 60 % of HBM; sparse row records (48 B per n_pad-wide
    destination row, ``csrc/ops/sparse_act.hip``) within 65 % (syn200: 2M x 91 KB = 182 GB of 288 GB; the learner
    needs < 40 GB).  ``mode`` auto: sparse only when ``eligible`` (native GPU learner, n_pad <= 238, critic
    first layer 64 wide) and the dense ring cannot hold ``cap`` transitions; "1" forces sparse where eligible,
    "0" dense.  Without HBM (CPU) the budget is 4 GB, dense."""
    obs_bytes = 4 * (2 * n_pad * n_obs + 4)
    dense_per = obs_bytes + action_bytes * action_dim
    sparse_per = obs_bytes + 48 * (action_dim // n_pad)
    if hbm <= 0:
        return False, dense_per, 4e9
    sparse = bool(eligible and mode != "0" and (mode == "1" or cap * dense_per > 0.6 * hbm))
    return (True, sparse_per, 0.65 * hbm) if sparse else (False, dense_per, 0.6 * hbm)


def _replay_hbm(device) -> float:
    """Device bytes the replay budget is a share of: this process's part of the GPU -- the total divided by the
    local ranks that share the device (a multi-process-per-GPU rehearsal), and never more than is free right now
    (another job on the card, or this rank's learner already allocated)."""
    if device.type != "cuda":
        return 0.0
    total = torch.cuda.get_device_properties(device).total_memory
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    per_dev = max(1, lw // max(1, torch.cuda.device_count()))
    free, _ = torch.cuda.mem_get_info(device)
    return float(min(total / per_dev, free))


class BatchedTrainer:
    """E lockstep environments on the device simulator + DDPG learner (one process per GPU)."""

    _AHEAD = 4  # steps the host may enqueue ahead of the simulator when hand-offs use sequence words

    def __init__(self, cfg: dict, sim: BatchedSimulator, tcfg: TrainerConfig, dist_info: Optional[DistInfo] = None,
                 network_schedule: Optional[Sequence[int]] = None, period: int = 0):
        self.cfg = cfg
        self.sim = sim
        self.t = tcfg
        self.dist = dist_info or DistInfo()
        self.device = sim.device
        self.E = sim.E
        self.graphs = GraphSet(sim.topologies, sim.n_pad, self.device)
        self.learner = DDPGLearner(cfg, sim.n_obs, sim.action_dim, self.graphs, sim.C, sim.F, self.device,
                                   self.dist, amp_bf16=tcfg.amp_bf16, seed=tcfg.seed)
        cap = tcfg.replay_capacity or min(int(cfg.get("mem_limit", 10000)) * self.E, tcfg.replay_cap_max)
        adt = torch.bfloat16 if self.learner.amp else torch.float32
        # Ring representation.  Dense: bf16 [A]-wide action rows.  Sparse (csrc/ops/sparse_act.hip): the
        # post-processed action as row records -- base value + <= 11 exceptions per n_pad-wide row, exact -- 48 B
        # per row instead of 2 n_pad B.  GSC_SPARSE_REPLAY=auto (default) picks sparse only when the dense ring
        # cannot hold the reference's min(mem_limit E, replay_cap_max) transitions in 60 % of HBM (config 5:
        # 2M x 720 KB; config 4's 2M x 45 KB fits dense, whose GEMMs are faster at small A); 1 forces it where
        # the native kernels apply (n_pad <= 238, critic first layer 64 wide), 0 disables it.
        R_rows = sim.action_dim // sim.n_pad
        hbm = _replay_hbm(self.device)
        eligible = bool(self.learner.native_ok and self.device.type == "cuda" and sim.n_pad <= 238
                        and self.learner.critic.mlp.layers[0].weight.shape[0] == 64)
        self.sparse_replay, per, budget = replay_plan(
            cap, sim.n_pad, sim.n_obs, sim.action_dim, torch.empty((), dtype=adt).element_size(), hbm, eligible,
            os.environ.get("GSC_SPARSE_REPLAY", "auto"))
        budget = tcfg.replay_bytes_max or budget
        cap = int(min(cap, budget // per))
        # on the GPU actions are stored in bf16: the critic consumes them as bf16 GEMM operands
        # (bf16 rows padded to 8 columns: 16-byte aligned operand rows for the native learner's GEMMs)
        self.replay = DeviceReplay(max(cap, self.E), sim.n_pad, sim.n_obs, sim.action_dim, self.device,
                                   action_dtype=adt, seed=tcfg.seed + 7919 * self.dist.rank,
                                   action_row_align=8 if adt == torch.bfloat16 else 1,
                                   sparse_rows=R_rows if self.sparse_replay else 0)
        self._pmask_ready = False   # this step's action producer wrote the simulator's destination bitsets
        self.batch_size = tcfg.batch_size or 100 * self.E
        self.learning_starts = (tcfg.learning_starts if tcfg.learning_starts is not None
                                else int(cfg.get("nb_steps_warmup_critic", 200)))
        self._warmup_steps = max(int(self.learning_starts), 1)
        self.rand_mu = float(cfg.get("rand_mu", 0.0))
        self.rand_sigma = float(cfg.get("rand_sigma", 0.3))
        self.sched_thr = schedule_threshold(cfg, sim.n_pad)  # reference 0.1 unless the config opts in
        self.global_step = 0
        self.episode = 0
        self.schedule = list(network_schedule) if network_schedule else [0]
        self.period = int(period) if period else 0
        self.sim.set_topologies(self.schedule[0])
        self._sched_idx = 0  # schedule entry last written to the simulator's next-reset topologies
        # acting actions are double-buffered by step parity and observations triple-buffered: with the
        # simulator overlapped, step t's replay insert runs after step t+1's simulator launch (off the
        # sim -> act -> sim critical path) and still reads step t's buffers, while the simulator writes
        # the observations of step t+2 straight into the third buffer (no copy on the critical path)
        first = self.sim.reset().clone()
        self._obs_bufs = [first, torch.empty_like(first), torch.empty_like(first)]
        self.topo = self.sim.topo_cur.to(torch.int64).clone()
        self.masks = self.learner.masks
        self._act_bufs = [torch.empty(self.E, sim.action_dim, device=self.device) for _ in range(2)]
        self._pending = None  # (obs, topo, act, out, sim event) of the last step, not yet in replay / metrics
        # recycled events of the act-on-simulator-stream chain (at most a few in flight)
        self._events = [torch.cuda.Event() for _ in range(6)] if self.device.type == "cuda" else []
        if self.device.type == "cuda":
            self.learner.enable_native_act(self.E)
        # device-side metric accumulators (read back only when logging)
        # [succ, drop, return of finished episodes, finished episodes] (one native kernel per step)
        self.acc = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.episode_returns: List[float] = []
        self.graphed = bool(tcfg.cuda_graphs and self.device.type == "cuda")
        self._batch = None
        self._topo_sink = None
        self._handoff = True
        self.sim_stream = self.learn_stream = None
        self.act_stream = None  # GSC_ACT_STREAM=1: the act path on an unmasked stream (every CU)
        self._words = 0         # signal words of the act <-> simulator hand-off (0: events)
        self._err_host = None   # the hand-off's wait-timed-out flag (mapped host word)
        self._ahead = collections.deque()  # simulator-done events of the last steps (run-ahead bound)
        self.sim_cus = 0
        if self.device.type == "cuda" and tcfg.overlap_sim:
            sim_cus = tcfg.sim_cus if tcfg.sim_cus >= 0 else self.auto_sim_cus(sim)
            if sim_cus > 0:
                # disjoint CU sets: the latency-bound simulator waves and the LDS-bound learner kernels
                # stop competing for the same CUs (scripts/cu_partition.py, profiles/)
                nat = sim.native
                n = nat.cu_count()
                k = max(8, min(int(sim_cus), n - 8))
                self.sim_cus = k
                small_env = (160 * 1024) // max(int(sim.ctx.lds_per_env), 1) >= 4
                sim_list = self.sim_cu_list(n, k, spread_default=small_env)
                rest = [c for c in range(n) if c not in set(sim_list)]
                self.sim_stream = torch.cuda.ExternalStream(nat.create_cu_masked_stream(sim_list),
                                                            device=self.device)
                # The learner stream is restricted to the complement, so no learner wave shares a SIMD
                # with a simulator wave -- when the simulator is the critical path (small topologies whose
                # envs pack three per CU: 103.6k vs 102.3k env-steps/s unmasked, 256 Abilene envs).  When
                # the learner is the longer chain (large graphs) the whole device serves it (--preset
                # syn50: 4.10k unmasked vs 3.56k masked).  GSC_LEARNER_MASK=0/1 forces either.
                mask_env = os.environ.get("GSC_LEARNER_MASK", "auto")
                small = (160 * 1024) // max(int(sim.ctx.lds_per_env), 1) >= 3
                learner_unmasked = mask_env == "0" or (mask_env == "auto" and not small)
                if learner_unmasked:
                    self.learn_stream = torch.cuda.Stream(self.device)
                else:
                    self.learn_stream = torch.cuda.ExternalStream(
                        nat.create_cu_masked_stream(rest), device=self.device)
                # The act path (actor forward + exploration of step t+1) sits between two simulator
                # steps, when the learner's CUs are idle too (update t done, update t+1 waits for it):
                # an unmasked stream gives it every CU.  Measured: syn50 19.41k -> 19.63k, syn200 5.08k ->
                # 5.13k (profiles/act_stream_ab.txt) and, since the simulator kernel's round-5 diet made
                # the headline simulator-bound with the learner finishing first, Abilene 114.4k -> 120.4k
                # (xcd-spread 64 simulator CUs).  GSC_ACT_STREAM=0 keeps it on the simulator's stream.
                act_env = os.environ.get("GSC_ACT_STREAM", "auto")
                if act_env != "0":
                    self.act_stream = torch.cuda.Stream(self.device)
                    # simulator <-> act hand-offs by sequence words (GSC_STREAM_VALUES=0: events).  Not under
                    # rocprofv3 counter collection: it serializes kernels, so a wait kernel would spin while its
                    # producer waits behind it (until the 10 s timeout)
                    counters = os.environ.get("ROCPROF_COUNTER_COLLECTION", "") not in ("", "0", "False", "false")
                    if os.environ.get("GSC_STREAM_VALUES", "1") != "0" and not counters and nat.stream_values_supported():
                        self._words = nat.alloc_signal_words(3)  # [simulator step done, act done, -]
                        self._seq = 0
                        weakref.finalize(self, nat.free_signal_words, self._words)
                        # wait-timed-out flag in mapped host memory: read every step without a sync; the host
                        # stays at most _AHEAD steps ahead of the simulator so a timeout fails the run promptly
                        hptr, self._err_dev = nat.alloc_host_word()
                        self._err_host = ctypes.c_uint32.from_address(hptr)
                        weakref.finalize(self, nat.free_host_word, hptr)
                # persistent GNN grids sized to the CUs free while the simulator runs (one full round)
                budget = int(os.environ.get("GSC_GNN_CU_BUDGET", str(n - k)))
                nat.gnn_set_cu_budget(budget)
                # the budget is process-wide state of the native module (overlap mode: work-queue grids, whose
                # per-workgroup gradient rows depend on the claim order): released with the trainer
                weakref.finalize(self, nat.gnn_set_cu_budget, 0)
            else:
                self.sim_stream = torch.cuda.Stream(self.device)

    @staticmethod
    def sim_cu_list(n: int, k: int, spread_default: bool = True) -> List[int]:
        """The simulator's CU-mask bits.  ``GSC_SIM_CU_LAYOUT=xcd``: k / 8 bits of every 32-bit block (the same
        CU count in each of MI355X's 8 XCDs); ``contig``: bits 0 .. k-1; auto (default): xcd for envs that
        pack four per CU (Abilene-class), else contig.  Measured round 5: 256 Abilene envs (4 per CU)
        standalone 64 contiguous bits 2.21 ms/step vs 64 spread 1.98 ms (the contiguous mask's waves stall
        on issue: SQ_WAIT_INST_ANY 2.85e7 vs 8.0e4 per dispatch at one wave per CU), bench 120.3k spread;
        syn50 23.8k contiguous vs 16.3k spread, syn200 5.24k vs 4.32k (their learner kernels need whole
        XCDs)."""
        layout = os.environ.get("GSC_SIM_CU_LAYOUT", "auto")
        if layout == "auto":
            layout = "xcd" if spread_default else "contig"
        if layout == "xcd" and n % 32 == 0 and k % (n // 32) == 0:
            per = k // (n // 32)
            return [c for c in range(n) if c % 32 < per]
        return list(range(k))

    @staticmethod
    def auto_sim_cus(sim) -> int:
        """CUs for one round of the simulator's env workgroups, at most 4 envs (waves) per CU with the
        default per-XCD spread mask (3 with contiguous mask bits), rounded up to a multiple of 8 (one per
        XCD block), capped at half the device.  Round 5, 256 Abilene envs: 64 spread CUs (8 per XCD)
        1.98 ms/step standalone vs 2.21 on 64 contiguous bits (2.06 on 96, 1.99 on 128 contiguous);
        bench 120.4k at 64 spread (with the act path on an unmasked stream), 113.7k at 96 contiguous.
        Earlier, on MI355X, 256 Abilene envs, 39.9 KB of LDS per env (env-steps/s, round 3): 64 CUs (two
        XCDs, 4 envs per CU) 113.3k; 96 CUs 111.0k; 128 CUs 96.4k (the learner becomes the longer
        chain); 72 / 80 / 88 / 112 CUs 71-84k (an XCD shared between simulator and learner); 32 CUs
        57.8k (two rounds).  Round 2, when an env took more LDS than 40 KB, 3 envs per CU (96 CUs) was
        the optimum."""
        nat = sim.native
        n = nat.cu_count()
        xcd = max(n // 8, 8)
        lds = max(int(sim.ctx.lds_per_env), 1)
        per_cu = max(1, min(4 if os.environ.get("GSC_SIM_CU_LAYOUT", "auto") != "contig" else 3, (160 * 1024) // lds))
        need = -(-sim.E // per_cu)
        # Mid-size topologies (33..64 nodes, two envs per CU by LDS) take one full round as well since round 5
        # (profiles/syn50_partition.txt, 256 syn50 envs at HEAD: 64 CUs 23.2k env-steps/s, 80 23.4k, 96 23.8k,
        # 128 24.0k, 160 23.5k, 192 22.9k).  In round 4, with a ~2x slower learner, half a round (64 CUs,
        # two simulator rounds) was best (16.4k vs 13.5k at 128).
        k = xcd * -(-need // xcd)
        return int(min(max(k, xcd), n // 2))

    def _schedule_next(self) -> None:
        """Network scheduler: topology used by the episode that starts after this step."""
        steps = self.sim.episode_steps
        if (self.global_step + 1) % steps == 0:
            nxt = self.episode + 1
            idx = (nxt // self.period) % len(self.schedule) if self.period else 0
            if idx != self._sched_idx:  # unchanged: the device table already holds it (no host copy)
                self.sim.set_topologies(self.schedule[idx])
                self._sched_idx = idx

    @property
    def obs(self) -> torch.Tensor:
        """Observation the next step acts on."""
        return self._obs_bufs[self.global_step % 3]

    @property
    def act_buf(self) -> torch.Tensor:
        return self._act_bufs[self.global_step & 1]

    def _record(self, obs, topo, act, out) -> None:
        """Replay insert + device-side metric accumulation of one finished step."""
        with trace_range("replay"):
            self.replay.add(obs, topo, act, out.reward, out.next_obs, out.done)
        st = out.stats
        self.replay.nat.step_metrics(self.device.type == "cuda", st.data_ptr(), st.shape[1], out.ep_return.data_ptr(),
                                     out.done.data_ptr(), self.E, self.acc.data_ptr(),
                                     torch.cuda.current_stream(self.device).cuda_stream
                                     if self.device.type == "cuda" else 0)

    def _event(self):
        return self._events.pop(0) if self._events else torch.cuda.Event()

    def _flush_pending(self) -> None:
        if self._pending is not None:
            p, self._pending = self._pending, None
            if p[4] is not None:  # simulator outputs produced on the simulator's stream
                torch.cuda.current_stream(self.device).wait_event(p[4])
                self._events.append(p[4])
            self._record(*p[:4])

    def _join(self) -> None:
        """Caller's stream waits for the trainer's streams; the next step re-syncs in the other direction."""
        if self.learn_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.learn_stream)
            self._handoff = True
        if self.sim_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.sim_stream)

    def flush(self) -> None:
        """Complete the deferred replay insert / metrics of the last step (before reading them)."""
        self._join()
        if self._pending is not None:
            if self.learn_stream is not None:
                self.learn_stream.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self.learn_stream):
                    self._flush_pending()
                torch.cuda.current_stream(self.device).wait_stream(self.learn_stream)
            else:
                self._flush_pending()

    def step(self) -> None:
        if self.learn_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            if self._handoff or not self.t.lazy_handoff:
                self.learn_stream.wait_stream(cur)
                self._handoff = False
            with torch.cuda.stream(self.learn_stream):
                self._step()
            if not self.t.lazy_handoff:
                cur.wait_stream(self.learn_stream)
        else:
            self._step()

    def _act(self, obs, topo, warm: bool, k: int) -> torch.Tensor:
        with trace_range("act"):
            mu = self.learner.act(obs, topo)
        with trace_range("explore"):
            # topologies beyond 64 nodes: the exploration kernel also writes the simulator's destination
            # bitsets from the rows it holds in registers (no second pass over the action block)
            pm = self.sim.pmask_target() if (mu.is_cuda and os.environ.get("GSC_EXPLORE_PMASK", "1") != "0") else None
            self._pmask_ready = pm is not None
            return explore_postprocess(mu, self.masks, self.sim.n_pad, warm, self.rand_mu, self.rand_sigma,
                                       seed=self.t.seed * 131 + self.dist.rank, step=self.global_step,
                                       threshold=self.sched_thr,
                                       out=self._act_bufs[k], topo=topo, pmask=pm)

    def _check_handoff(self) -> None:
        """Fail the run if a sequence-word wait timed out: wait for the simulator of _AHEAD steps ago (already done
        in steady state: the GPU has that many steps queued), then read the mapped host flag."""
        while len(self._ahead) >= self._AHEAD:
            self._ahead.popleft().synchronize()
        if self._err_host is not None and self._err_host.value:
            raise RuntimeError(f"act / simulator hand-off: a stream waited {self.t.handoff_timeout_s:g} s for its "
                               f"sequence word (step {self.global_step}); the run is aborted, its replay data after "
                               "the timeout is invalid")

    def _step(self) -> None:
        if self._words:
            self._check_handoff()
        warm = self.global_step < self.learning_starts
        k = self.global_step & 1
        obs, topo = self._obs_bufs[self.global_step % 3], self.topo
        obs_next = self._obs_bufs[(self.global_step + 1) % 3]
        episode_end = (self.global_step + 1) % self.sim.episode_steps == 0
        train = self.global_step >= self.learning_starts - 1 and (len(self.replay) > 0 or self._pending is not None)
        overlap = self.sim_stream is not None and train
        main = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        new_topo = None
        if overlap and self.t.act_on_sim_stream:
            # act(t) -> explore(t) -> simulator(t) in order on the simulator's stream, after everything the
            # learner's stream holds so far (update t-1 wrote the actor weights; replay inserts read the
            # buffers this step reuses).  The learner's replay insert of step t-1 and update t wait for the
            # act only (the update rewrites the actor weights), so they run concurrently with simulator(t).
            self.sim_stream.wait_stream(main)
            if self.act_stream is not None and self._words:
                # sequence words instead of events on the chain simulator(t-1) -> act(t) -> simulator(t): the
                # act waits for the learner's stream (actor weights, by event: that work finished long before)
                # and for the simulator's word; the simulator for the act's word (csrc/ops/streams.hip,
                # profiles/handoff_ab.txt)
                nat, seq, sim_word, act_word = self.sim.native, self._seq, self._words, self._words + 4
                err, tmo = self._err_dev, float(self.t.handoff_timeout_s)
                self.act_stream.wait_stream(main)
                if seq > 0:
                    nat.wait_word(self.act_stream.cuda_stream, sim_word, seq, err, tmo)
                with torch.cuda.stream(self.act_stream):
                    act = self._act(obs, topo, warm, k)
                    # the signal right behind the last act kernel: an event record between them costs the
                    # chain ~7 us of marker processing (rocprofv3 trace)
                    nat.signal_word(self.act_stream.cuda_stream, act_word, seq + 1)
                    ev_act = self._event()
                    ev_act.record(self.act_stream)
                nat.wait_word(self.sim_stream.cuda_stream, act_word, seq + 1, err, tmo)
            elif self.act_stream is not None:
                self.act_stream.wait_stream(self.sim_stream)
                with torch.cuda.stream(self.act_stream):
                    act = self._act(obs, topo, warm, k)
                    ev_act = self._event()
                    ev_act.record(self.act_stream)
                self.sim_stream.wait_event(ev_act)
            with torch.cuda.stream(self.sim_stream):
                if self.act_stream is None:
                    act = self._act(obs, topo, warm, k)
                    ev_act = self._event()
                    ev_act.record(self.sim_stream)
                self._schedule_next()
                out = self.sim.step(act, buffer_set=k, obs_out=obs_next, pmask_ready=self._pmask_ready)
                if self.act_stream is not None and self._words:  # right behind the simulator kernel
                    self.sim.native.signal_word(self.sim_stream.cuda_stream, self._words, self._seq + 1)
                    self._seq += 1
                    ahead = torch.cuda.Event()
                    ahead.record(self.sim_stream)
                    self._ahead.append(ahead)
                ev_sim = self._event()
                ev_sim.record(self.sim_stream)
                if episode_end:
                    new_topo = self.sim.topo_next.to(torch.int64).clone()
            main.wait_event(ev_act)
            self._events.append(ev_act)
            self._flush_pending()
            with trace_range("learn"):
                self._learn()
            self._pending = (obs, topo, act, out, ev_sim)
        elif overlap:
            act = self._act(obs, topo, warm, k)
            self._schedule_next()
            # simulator kernel (one wave per env) runs concurrently with the previous step's replay
            # insert and the learner update, which samples transitions up to the previous step
            self.sim_stream.wait_stream(main)
            with torch.cuda.stream(self.sim_stream):
                out = self.sim.step(act, buffer_set=k, obs_out=obs_next, pmask_ready=self._pmask_ready)
            self._flush_pending()
            with trace_range("learn"):
                self._learn()
            main.wait_stream(self.sim_stream)
            self._pending = (obs, topo, act, out, None)
        else:
            act = self._act(obs, topo, warm, k)
            self._schedule_next()
            self._flush_pending()
            with trace_range("sim"):
                out = self.sim.step(act, buffer_set=k, obs_out=obs_next, pmask_ready=self._pmask_ready)
            self._record(obs, topo, act, out)
            if train:
                with trace_range("learn"):
                    self._learn()
        if episode_end:
            self.episode += 1
            self.topo = new_topo if new_topo is not None else self.sim.topo_next.to(torch.int64).clone()
        self.global_step += 1
        # pool overflow (flows / processes / events dropped) fails the run at the latest at the end of
        # the episode it happened in (one flag read per episode), or every check_every steps
        if episode_end or (self.t.check_every and self.global_step % self.t.check_every == 0):
            if overlap and self.t.act_on_sim_stream:
                main.wait_stream(self.sim_stream)
            self.sim.check_flags()
            self.replay.check_sparse()

    def _learn(self) -> None:
        if _DIAG_NO_LEARN:  # diagnostics only (never in bench numbers): measures the act + sim chain alone
            return
        for _ in range(self.t.updates_per_step):
            if self.graphed or self.replay.sparse_rows:
                if self._batch is None:
                    B = self.batch_size
                    fused = self.fused_action_gather()
                    self._batch = self.replay.empty_batch(B, actions=not fused)
                    out = self._batch
                    if fused:  # the critic's action GEMMs read the sampled ring rows in place
                        nu = self.learner.native_update(B)
                        nu.act_rows = self.replay.indices(B)
                        if self.replay.sparse_rows:
                            nu.set_sparse(self.replay.actions, self.replay.sparse_rows, self.replay.n_pad)
                    sink = self._topo_sink = self.learner.topo32_buffer(B)
                    self._sampler = lambda: self.replay.sample(B, out=out, topo32=sink, actions=not fused)
                if self.graphed:
                    self.learner.update_graphed(self._batch, pre=self._sampler, topo_ready=self._topo_sink is not None)
                else:
                    self._sampler()
                    self.learner.update(self._batch)
            else:
                self.learner.update(self.replay.sample(self.batch_size))

    def fused_action_gather(self) -> bool:
        """Replayed actions read in place by the native learner's GEMMs (row-indexed operands) instead of
        gathered into a [B, A] batch: on by default once that batch copy exceeds 256 MB (50/200-node
        topologies: 1.2 / 18 GB at B = 25,600); GSC_FUSED_GATHER=0/1 forces it."""
        if self.replay.sparse_rows:
            return True   # sparse records are only ever read in place
        if not (self.learner.native_ok and self.replay.actions.dtype == torch.bfloat16):
            return False
        env = os.environ.get("GSC_FUSED_GATHER")
        if env is not None:
            return env == "1"
        return self.batch_size * self.replay.action_cols * 2 > (256 << 20)

    def metrics(self, reset: bool = True) -> dict:
        self.flush()
        vals = self.acc.clone()
        if self.dist.enabled:
            allreduce_sum_(vals)
        s, d, r, e = [float(v) for v in vals.cpu()]
        if reset:
            self.acc.zero_()
        out = {"success_ratio": s / (s + d) if s + d > 0 else 0.0, "succ": s, "drop": d, "episodes": e,
               "mean_episode_return": r / e if e > 0 else float("nan")}
        for k, v in self.learner.last.items():
            out[k] = float(v)
        return out

    def replay_bytes(self) -> int:
        r = self.replay
        return sum(t[:len(r)].numel() * t.element_size() for t in (r.obs, r.next_obs, r.topo, r.actions, r.rewards,
                                                                  r.dones))

    def state_dict(self, include_replay: bool = True) -> dict:
        self.flush()
        sd = {"learner": self.learner.state_dict(), "global_step": self.global_step, "episode": self.episode,
              "sim_states": self.sim.states.cpu(), "obs": self.obs.cpu(), "topo": self.topo.cpu(),
              "rng": self.replay.rng_state()}
        if include_replay:
            sd["replay"] = self.replay.state_dict()
        return sd

    def load_state_dict(self, sd: dict) -> None:
        self._join()
        self.learner.load_state_dict(sd["learner"])
        self.global_step = int(sd["global_step"])
        self.episode = int(sd["episode"])
        self.sim.states.copy_(sd["sim_states"].to(self.device))
        self._pending = None
        self.obs.copy_(sd["obs"].to(self.device))
        self.topo = sd["topo"].to(self.device)
        if "replay" in sd:
            self.replay.load_state_dict(sd["replay"])
        self.replay.set_rng_state(sd["rng"])
        if "replay" not in sd:  # checkpoint without the replay ring: resume refills it for a full warm-up
            self.replay.pos, self.replay.full = 0, False
            self.replay.state[:2] = 0
            self.learning_starts = self.global_step + self._warmup_steps

    def reseed(self, seed: int) -> None:
        """Fresh rank-local randomness (resume of a checkpoint without this rank's state): new
        simulator Philox keys (all envs restart their episode) and a new replay sampler stream."""
        self._join()
        g = np.random.default_rng(seed)
        self.sim.seeds.copy_(torch.from_numpy(g.integers(1, 2**31 - 1, size=self.E).astype(np.uint32)
                                              .view(np.int32)).to(self.device))
        self.sim.set_topologies(self.topo.to(torch.int32))
        self._sched_idx = None  # per-env table written directly: the next scheduled entry is rewritten
        self._obs_bufs[self.global_step % 3].copy_(self.sim.reset())
        self.replay.reseed(int(seed) * 7919 + self.global_step)
