"""Agent base class (reference ``src/rlsp/agents/rlsp_agent.py``: an empty ``RLSPAgent`` stub).

Here it fixes the interface every agent exposes to ``main.py`` / ``inference.py``."""
from __future__ import annotations

from abc import ABC, abstractmethod


class RLSPAgent(ABC):
    @abstractmethod
    def train(self, episodes: int) -> dict:
        """Train for ``episodes`` episodes (per environment)."""

    @abstractmethod
    def predict(self, obs, topo=None):
        """Greedy action for an observation."""

    @abstractmethod
    def test(self, episode_steps=None, seed=None) -> dict:
        """One greedy episode on the inference network (test-mode simulator outputs)."""

    @abstractmethod
    def save_checkpoint(self, path: str) -> None: ...

    @abstractmethod
    def load_checkpoint(self, path: str) -> None: ...
