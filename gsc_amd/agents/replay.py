"""Replay buffers.

``DeviceReplay`` keeps transitions in HBM as structure-of-arrays tensors (node features, topology
id, post-processed action, reward, done) — masks and edge lists are derived from the topology id
instead of being stored per transition.  Inserts and samples are native kernels (Philox index
draw + row gathers, ``csrc/ops/replay.hip``) with the ring cursor on the device, so the learner
never touches the host and sampling is captured with the update.  Sampling follows the
reference ``GraphReplayBuffer.sample`` (``buffer.py:56-62``): uniform over the filled part, and
once full the slot at the write position (the next one to be overwritten) is excluded.

``GraphReplayBuffer`` is the host-side ring used by the reference-equivalent single-env agent.
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import numpy as np
import torch


class Batch(NamedTuple):
    obs: torch.Tensor        # [B, n_pad, F]
    topo: torch.Tensor       # [B] int64
    actions: torch.Tensor    # [B, A] (bf16 on the GPU, float32 on CPU); rows may carry zero padding
                             # columns beyond A (DeviceReplay action_row_align): use actions[:, :A]
    rewards: torch.Tensor    # [B]
    next_obs: torch.Tensor   # [B, n_pad, F]
    dones: torch.Tensor      # [B]


class DeviceReplay:
    """Structure-of-arrays ring in HBM (or host memory on CPU) driven by the native replay kernels
    (``csrc/ops/replay.hip``): the write cursor and the sampler's draw counter live in a device int64
    ``state`` tensor ``[pos, full, draws, -]``, so :meth:`add` and :meth:`sample` are fixed-argument
    kernel launches that run inside captured HIP graphs.  Indices come from Philox4x32-10 keyed by
    ``seed`` (rank-specific) and the draw counter -- the same stream on the host path."""

    def __init__(self, capacity: int, n_pad: int, n_obs: int, action_dim: int, device,
                 action_dtype=torch.float32, seed: int = 0, action_row_align: int = 1, sparse_rows: int = 0):
        """``sparse_rows`` = R > 0 (GPU): actions are stored as R row records of n_pad destinations each
        (``csrc/ops/sparse_act.hip``: base value + <= 11 exceptions, exactly the bf16 row), ~8x smaller than
        dense bf16 at 200-node topologies; ``actions`` is then the int32 [capacity, R, 12] record ring."""
        from gsc_amd.native import load as load_native
        self.nat = load_native()
        self.capacity = int(capacity)
        dev = torch.device(device)
        self.device = dev
        self.is_dev = dev.type == "cuda"
        self.obs = torch.zeros((self.capacity, n_pad, n_obs), dtype=torch.float32, device=dev)
        self.next_obs = torch.zeros_like(self.obs)
        self.topo = torch.zeros(self.capacity, dtype=torch.int64, device=dev)
        # ``action_row_align``: ring (and sampled batch) rows padded to a multiple of that many columns
        # (zeros), so every action row starts 16-byte aligned for the native learner's vector loads
        # (A % 8 != 0 at 50-node topologies); consumers use ``actions[:, :action_dim]``
        self.action_dim = int(action_dim)
        al = max(1, int(action_row_align))
        self.action_cols = -(-self.action_dim // al) * al
        self.sparse_rows = int(sparse_rows)
        self.n_pad = int(n_pad)
        if self.sparse_rows:
            assert self.is_dev and self.sparse_rows * self.n_pad == self.action_dim, "sparse rows: R * n_pad == A"
            self.actions = torch.zeros((self.capacity, self.sparse_rows, self.nat.SPARSE_ACT_WORDS), dtype=torch.int32,
                                       device=dev)
            self.sparse_bad = torch.zeros(1, dtype=torch.int32, device=dev)   # rows that did not compress
        else:
            self.actions = torch.zeros((self.capacity, self.action_cols), dtype=action_dtype, device=dev)
        self.rewards = torch.zeros(self.capacity, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(self.capacity, dtype=torch.float32, device=dev)
        self.state = torch.zeros(4, dtype=torch.int64, device=dev)   # pos, full, draws, -
        self.seed = int(seed) & 0xffffffff
        self.pos = 0        # host mirrors of the device cursor (deterministic: E rows per add)
        self.full = False
        self._idx = {}

    def __len__(self) -> int:
        return self.capacity if self.full else self.pos

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.is_dev else 0

    def reseed(self, seed: int) -> None:
        self.seed = int(seed) & 0xffffffff
        self.state[2] = 0

    @torch.no_grad()
    def add(self, obs, topo, actions, rewards, next_obs, dones) -> None:
        """Insert E rows at the device cursor.  ``dones``: uint8/bool/float [E]."""
        E = obs.shape[0]
        if E > self.capacity:
            raise ValueError("batch larger than replay capacity")
        nat, s, dev, cap, st = self.nat, self._stream(), self.is_dev, self.capacity, self.state.data_ptr()
        obs, next_obs = obs.contiguous().float(), next_obs.contiguous().float()
        topo = topo.to(torch.int64).contiguous()
        rewards = rewards.contiguous().float()
        ob = obs[0].numel() * 4
        cols = [(obs.data_ptr(), self.obs.data_ptr(), ob, 0, 0),
                (next_obs.data_ptr(), self.next_obs.data_ptr(), ob, 0, 0),
                (topo.data_ptr(), self.topo.data_ptr(), 8, 0, 0), (rewards.data_ptr(), self.rewards.data_ptr(), 4, 0, 0)]
        A, Ap = self.action_dim, self.action_cols
        if self.sparse_rows:
            # compressed rows at the cursor, before the column insert advances it
            a = actions.contiguous().float()
            nat.sparse_compress(a.data_ptr(), a.stride(0), E, self.sparse_rows, self.n_pad, self.actions.data_ptr(), st,
                                cap, self.sparse_bad.data_ptr(), s)
        elif self.actions.dtype == torch.bfloat16 and actions.dtype == torch.float32:
            a = actions.contiguous()
            cols.append((a.data_ptr(), self.actions.data_ptr(), A, 1, Ap))
        else:
            a = actions.to(self.actions.dtype).contiguous()
            es = a.element_size()
            cols.append((a.data_ptr(), self.actions.data_ptr(), A * es, 0, Ap * es))
        if dones.dtype in (torch.uint8, torch.bool):
            d = dones.contiguous().view(torch.uint8)
            cols.append((d.data_ptr(), self.dones.data_ptr(), 1, 2, 0))
        else:
            d = dones.contiguous().float()
            cols.append((d.data_ptr(), self.dones.data_ptr(), 4, 0, 0))
        # every column in one kernel, then the cursor advance (csrc/ops/replay.hip insert_cols_kernel)
        nat.replay_insert_cols(dev, st, E, cap, cols, s)
        new = self.pos + E
        if new >= self.capacity:
            self.full = True
        self.pos = new % self.capacity

    @torch.no_grad()
    def indices(self, batch_size: int) -> torch.Tensor:
        """The (static) int32 row-index buffer a sample of ``batch_size`` writes."""
        B = int(batch_size)
        idx = self._idx.get(B)
        if idx is None:
            idx = self._idx[B] = torch.empty(B, dtype=torch.int32, device=self.device)
        return idx

    def sample(self, batch_size: int, out: Optional[Batch] = None, topo32: Optional[torch.Tensor] = None,
               actions: bool = True) -> Batch:
        """Uniform sample (reference buffer.py:56-62); with ``out`` the rows are gathered into those
        (static) buffers -- graph-capturable.  ``topo32`` (int32 [B]) also receives the sampled
        topology ids (the native learner's kernels take int32).  ``actions=False``: the action column is
        not gathered -- the native learner reads the sampled ring rows in place through
        :meth:`indices` (row-indexed GEMM operands); ``out.actions`` is then the ring itself."""
        if len(self) == 0:
            raise RuntimeError("cannot sample from an empty replay buffer")
        B = int(batch_size)
        idx = self.indices(B)
        if out is None:
            out = self.empty_batch(B, actions=actions)
        nat, s, dev = self.nat, self._stream(), self.is_dev
        cols = []
        if self.sparse_rows and actions:
            raise ValueError("a sparse action ring is read in place (sample(actions=False))")
        for src, dst in zip((self.obs, self.topo, self.actions, self.rewards, self.next_obs, self.dones), out):
            if src is self.actions and not actions:
                assert dst is self.actions
                continue
            assert dst.is_contiguous() and dst.shape[0] == B and dst.dtype == src.dtype
            cols.append((src.data_ptr(), dst.data_ptr(), src[0].numel() * src.element_size(), 0))
        if topo32 is not None:
            assert topo32.dtype == torch.int32 and topo32.is_contiguous() and topo32.numel() == B
            cols.append((self.topo.data_ptr(), topo32.data_ptr(), 8, 3))
        # Philox indices, then every column in one gather kernel (csrc/ops/replay.hip gather_cols_kernel)
        nat.replay_sample_cols(dev, self.state.data_ptr(), self.seed, B, self.capacity, idx.data_ptr(), cols, s)
        return out

    def last_indices(self, batch_size: int) -> torch.Tensor:
        return self._idx[int(batch_size)]

    def empty_batch(self, batch_size: int, actions: bool = True) -> Batch:
        """Static batch buffers (for :meth:`sample` ``out=`` and HIP-graph replay); ``actions=False``: the
        batch's action slot is the ring itself (rows addressed through :meth:`indices`)."""
        mk = lambda t: torch.empty((batch_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
        return Batch(mk(self.obs), mk(self.topo), mk(self.actions) if actions else self.actions, mk(self.rewards),
                     mk(self.next_obs), mk(self.dones))

    def rng_state(self) -> torch.Tensor:
        return torch.cat([self.state.cpu(), torch.tensor([self.seed], dtype=torch.int64)])

    def set_rng_state(self, t: torch.Tensor) -> None:
        t = t.to(torch.int64).cpu()
        if t.numel() != 5:
            raise ValueError("replay sampler state: expected [pos, full, draws, -, seed]")
        self.state.copy_(t[:4].to(self.device))
        self.seed = int(t[4])

    def check_sparse(self) -> None:
        """Raise if a stored row did not fit the sparse record (not a post-processed action row)."""
        if self.sparse_rows and int(self.sparse_bad.item()) > 0:
            raise RuntimeError(f"{int(self.sparse_bad.item())} replayed action rows exceeded the sparse record's "
                               "exceptions (post-processed rows hold <= 11); run with GSC_SPARSE_REPLAY=0")

    def dense_actions(self, rows: torch.Tensor) -> torch.Tensor:
        """bf16 [len(rows), A] actions of ring rows (sparse rings decompressed; tests and checkpoints)."""
        if not self.sparse_rows:
            return self.actions[rows.long(), :self.action_dim].to(torch.bfloat16)
        return decompress_actions(self.actions[rows.long()], self.n_pad)

    def state_dict(self) -> dict:
        n = len(self)
        acts = self.actions[:n].cpu() if self.sparse_rows else self.actions[:n, :self.action_dim].cpu()
        return {"pos": self.pos, "full": self.full, "obs": self.obs[:n].cpu(), "next_obs": self.next_obs[:n].cpu(),
                "topo": self.topo[:n].cpu(), "actions": acts,
                "rewards": self.rewards[:n].cpu(),
                "dones": self.dones[:n].cpu()}

    def load_state_dict(self, sd: dict) -> None:
        n = sd["obs"].shape[0]
        for k in ("obs", "next_obs", "topo", "rewards", "dones"):
            getattr(self, k)[:n].copy_(sd[k].to(self.device))
        if self.sparse_rows:
            if sd["actions"].dim() != 3:
                raise ValueError("checkpoint holds dense replay actions; this ring stores sparse rows")
            self.actions[:n].copy_(sd["actions"].to(self.device))
        else:
            self.actions[:n, :self.action_dim].copy_(sd["actions"].to(self.device))
        self.pos, self.full = int(sd["pos"]), bool(sd["full"])
        self.state[0] = self.pos
        self.state[1] = int(self.full)


def decompress_actions(rec: torch.Tensor, n_pad: int) -> torch.Tensor:
    """Dense bf16 [..., R * n_pad] actions from sparse row records [..., R, 12] (int32): every destination takes
    the row's base value, listed exceptions their own (the reference for ``csrc/ops/sparse_act.hip``)."""
    rec = rec.to(torch.int64) & 0xffffffff
    head = rec[..., 0]
    base = (head & 0xffff).to(torch.int32)
    cnt = (head >> 16) & 0xffff
    bits = base.unsqueeze(-1).expand(*base.shape, n_pad + 1).clone()   # column n_pad: sink of unused slots
    slots = rec[..., 1:]
    k = torch.arange(slots.shape[-1], device=rec.device)
    valid = k < cnt.unsqueeze(-1)
    idx = torch.where(valid, (slots & 0xffff).clamp(max=n_pad - 1), torch.full_like(slots, n_pad))
    val = ((slots >> 16) & 0xffff).to(torch.int32)
    bits.scatter_(-1, idx, val)
    f = (bits[..., :n_pad].to(torch.int32) << 16).view(torch.float32)
    return f.reshape(*f.shape[:-2], -1).to(torch.bfloat16)


class GraphReplayBuffer:
    """Host ring buffer of single-graph transitions (reference ``src/rlsp/agents/buffer.py``)."""

    def __init__(self, buffer_size: int, action_dim: int, n_pad: int, n_obs: int, rng: Optional[np.random.RandomState] = None):
        self.buffer_size = int(buffer_size)
        self.dones = np.ones(self.buffer_size, np.float32)
        self.rewards = np.zeros(self.buffer_size, np.float32)
        self.actions = np.zeros((self.buffer_size, action_dim), np.float32)
        self.obs = np.zeros((self.buffer_size, n_pad, n_obs), np.float32)
        self.next_obs = np.zeros_like(self.obs)
        self.topo = np.zeros(self.buffer_size, np.int64)
        self.pos = 0
        self.full = False
        self.rng = rng if rng is not None else np.random

    def add(self, obs_x: np.ndarray, topo: int, next_x: np.ndarray, action, reward, done) -> None:
        n = obs_x.shape[0]
        self.obs[self.pos] = 0
        self.obs[self.pos, :n] = obs_x
        self.next_obs[self.pos] = 0
        self.next_obs[self.pos, :next_x.shape[0]] = next_x
        self.topo[self.pos] = topo
        self.actions[self.pos] = action
        self.rewards[self.pos] = reward
        self.dones[self.pos] = done
        self.pos += 1
        if self.pos == self.buffer_size:
            self.pos = 0
            self.full = True

    def __len__(self):
        return self.buffer_size if self.full else self.pos

    def sample(self, batch_size: int, device="cpu") -> Batch:
        if self.full:
            idx = (self.rng.randint(1, self.buffer_size, size=batch_size) + self.pos) % self.buffer_size
        else:
            idx = self.rng.randint(0, self.pos, size=batch_size)
        t = lambda a: torch.from_numpy(a[idx]).to(device)
        return Batch(t(self.obs), t(self.topo), t(self.actions), t(self.rewards), t(self.next_obs), t(self.dones))
