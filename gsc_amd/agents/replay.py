"""Replay buffers.

``DeviceReplay`` keeps transitions in HBM as structure-of-arrays tensors (node features, topology
id, post-processed action, reward, done) — masks and edge lists are derived from the topology id
instead of being stored per transition.  Adds are one indexed copy of E rows; sampling is a
device ``randint`` + gather, so the learner never touches the host.  Sampling follows the
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
    actions: torch.Tensor    # [B, A] (bf16 on the GPU, float32 on CPU)
    rewards: torch.Tensor    # [B]
    next_obs: torch.Tensor   # [B, n_pad, F]
    dones: torch.Tensor      # [B]


class DeviceReplay:
    def __init__(self, capacity: int, n_pad: int, n_obs: int, action_dim: int, device,
                 action_dtype=torch.float32, seed: int = 0):
        self.capacity = int(capacity)
        dev = torch.device(device)
        self.device = dev
        self.obs = torch.zeros((self.capacity, n_pad, n_obs), dtype=torch.float32, device=dev)
        self.next_obs = torch.zeros_like(self.obs)
        self.topo = torch.zeros(self.capacity, dtype=torch.int64, device=dev)
        self.actions = torch.zeros((self.capacity, action_dim), dtype=action_dtype, device=dev)
        self.rewards = torch.zeros(self.capacity, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(self.capacity, dtype=torch.float32, device=dev)
        self.pos = 0
        self.full = False
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)

    def __len__(self) -> int:
        return self.capacity if self.full else self.pos

    @torch.no_grad()
    def add(self, obs, topo, actions, rewards, next_obs, dones) -> None:
        E = obs.shape[0]
        if E > self.capacity:
            raise ValueError("batch larger than replay capacity")
        idx = (torch.arange(E, device=self.device) + self.pos) % self.capacity
        self.obs.index_copy_(0, idx, obs)
        self.next_obs.index_copy_(0, idx, next_obs)
        self.topo.index_copy_(0, idx, topo.to(torch.int64))
        self.actions.index_copy_(0, idx, actions.to(self.actions.dtype))
        self.rewards.index_copy_(0, idx, rewards.float())
        self.dones.index_copy_(0, idx, dones.float())
        new = self.pos + E
        if new >= self.capacity:
            self.full = True
        self.pos = new % self.capacity

    @torch.no_grad()
    def sample(self, batch_size: int, out: Optional[Batch] = None) -> Batch:
        """Uniform sample; with ``out`` the rows are gathered into those (static) buffers."""
        if self.full:
            idx = (torch.randint(1, self.capacity, (batch_size,), device=self.device, generator=self.gen)
                   + self.pos) % self.capacity
        else:
            if self.pos == 0:
                raise RuntimeError("cannot sample from an empty replay buffer")
            idx = torch.randint(0, self.pos, (batch_size,), device=self.device, generator=self.gen)
        if out is None:
            return Batch(self.obs.index_select(0, idx), self.topo.index_select(0, idx),
                         self.actions.index_select(0, idx), self.rewards.index_select(0, idx),
                         self.next_obs.index_select(0, idx), self.dones.index_select(0, idx))
        for src, dst in zip((self.obs, self.topo, self.actions, self.rewards, self.next_obs, self.dones), out):
            torch.index_select(src, 0, idx, out=dst)
        return out

    def empty_batch(self, batch_size: int) -> Batch:
        """Static batch buffers (for :meth:`sample` ``out=`` and HIP-graph replay)."""
        mk = lambda t: torch.empty((batch_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
        return Batch(mk(self.obs), mk(self.topo), mk(self.actions), mk(self.rewards), mk(self.next_obs),
                     mk(self.dones))

    def state_dict(self) -> dict:
        n = len(self)
        return {"pos": self.pos, "full": self.full, "obs": self.obs[:n].cpu(), "next_obs": self.next_obs[:n].cpu(),
                "topo": self.topo[:n].cpu(), "actions": self.actions[:n].cpu(), "rewards": self.rewards[:n].cpu(),
                "dones": self.dones[:n].cpu()}

    def load_state_dict(self, sd: dict) -> None:
        n = sd["obs"].shape[0]
        for k in ("obs", "next_obs", "topo", "actions", "rewards", "dones"):
            getattr(self, k)[:n].copy_(sd[k].to(self.device))
        self.pos, self.full = int(sd["pos"]), bool(sd["full"])


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
