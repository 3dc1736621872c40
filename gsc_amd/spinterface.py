"""Simulator <-> algorithm API (reference: ``spinterface/spinterface.py``).

These three classes are the stable public contract between the RL layer and
any simulator backend (the scalar CPU oracle, the dummy backend, or one env of
the batched device simulator).
"""
from __future__ import annotations

from abc import ABC, abstractmethod


class SimulatorAction:
    """Placement ``{node: [sf, ...]}`` and scheduling ``{node: {sfc: {sf: {dst_node: weight}}}}``.

    The scheduling table must list every destination node (zeros included); the
    weights of one ``(node, sfc, sf)`` entry are expected to sum to one.
    """

    def __init__(self, placement: dict, scheduling: dict):
        self.placement = placement
        self.scheduling = scheduling

    def __repr__(self):
        return f"SimulatorAction(placement={self.placement!r}, scheduling={self.scheduling!r})"


class SimulatorState:
    """Network view returned by ``init``/``apply``.

    ``network``: ``{'nodes': [{'id', 'resource', 'used_resources'}], 'edges': [{'src', 'dst', 'delay',
    'data_rate', 'used_data_rate'}]}``; ``placement``; ``sfcs``; ``service_functions``; ``traffic``
    ``{node: {sfc: {sf: requested_rate}}}`` and ``network_stats`` (success/drop counters, delays).
    """

    def __init__(self, network, placement, sfcs, service_functions, traffic, network_stats):
        self.network = network
        self.placement = placement
        self.sfcs = sfcs
        self.service_functions = service_functions
        self.traffic = traffic
        self.network_stats = network_stats

    def __repr__(self):
        return (f"SimulatorState(nodes={len(self.network.get('nodes', []))}, "
                f"edges={len(self.network.get('edges', []))}, stats={self.network_stats})")


class SimulatorInterface(ABC):
    def __init__(self, test_mode: bool = False):
        self.test_mode = test_mode

    @abstractmethod
    def init(self, seed: int) -> SimulatorState:
        """Create a new simulation (episode) with ``seed`` and return the initial state."""

    @abstractmethod
    def apply(self, actions: SimulatorAction) -> SimulatorState:
        """Apply placement + scheduling, advance one run window, return the new state."""

    def get_active_ingress_nodes(self):
        return []
