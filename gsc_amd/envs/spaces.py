"""Minimal gym-compatible spaces (gym is not a dependency of this framework)."""
from __future__ import annotations

from typing import Dict as TDict, Optional

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None, seed: Optional[int] = None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed: Optional[int] = None):
        self.np_random = np.random.default_rng(seed)
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        if shape is None:
            shape = np.shape(low)
        super().__init__(shape, dtype, seed)
        self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self.np_random.integers(self.low, self.high + 1, size=self.shape).astype(self.dtype)
        return self.np_random.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Dict(Space):
    def __init__(self, spaces: TDict[str, Space], seed=None):
        super().__init__(None, None, seed)
        self.spaces = dict(spaces)

    def __getitem__(self, key):
        return self.spaces[key]

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def __repr__(self):
        return f"Dict({self.spaces})"
