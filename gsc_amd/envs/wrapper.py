"""Action/observation codec between flat arrays and the simulator API.

Reference: ``src/rlsp/envs/simulator_wrapper.py``.
* ``apply``: takes the ``[:n, :, :, :n]`` block of the padded action, builds
  ``scheduling[src][sfc][sf][dst]``, derives the placement by following
  positive weights from every active ingress node along the chain, and calls
  ``simulator.apply``.
* graph observation (``_parse_state_as_graph``): per-node features in
  ``observation_space`` order — ingress traffic, node load, node capacity —
  each max-normalised with ``+1e-3``; bidirectional edge index; action mask.
* flat observation and node-permutation helpers (reference flat mode).
"""
from __future__ import annotations

import logging
from typing import Tuple

import numpy as np
import torch

from gsc_amd.spinterface import SimulatorAction, SimulatorState
from .graph import GraphObs
from .limits import EnvironmentLimits

logger = logging.getLogger(__name__)


def node_features(state: SimulatorState, node_map: dict, observations_space) -> np.ndarray:
    """``[n, F]`` float32 features in ``observations_space`` order (simulator_wrapper.py:255-294)."""
    n = len(state.network["nodes"])
    cols = []
    if "ingress_traffic" in observations_space:
        t = np.zeros(n, dtype=np.float32)
        for node, sfc_dict in state.traffic.items():
            for sfc, sf_dict in sfc_dict.items():
                t[node_map[node]] = sf_dict[state.sfcs[sfc][0]]
        cols.append(np.clip(t / (np.max(t) + 1e-3), 0, 1))
    if "node_load" in observations_space:
        u = np.zeros(n, dtype=np.float32)
        for node in state.network["nodes"]:
            cap = node["resource"]
            usage = sum(state.network_stats["run_total_processed_traffic"][node["id"]].values())
            u[node_map[node["id"]]] = 1 if cap == 0 else usage / cap
        cols.append(np.clip(u / (np.max(u) + 1e-3), 0, 1))
    if "node_cap" in observations_space:
        c = np.zeros(n, dtype=np.float32)
        for node in state.network["nodes"]:
            c[node_map[node["id"]]] = node["resource"]
        cols.append(np.clip(c / (np.max(c) + 1e-3), 0, 1))
    return np.stack(cols, axis=1).astype(np.float32) if cols else np.zeros((n, 0), np.float32)


class SimulatorWrapper:
    def __init__(self, simulator, env_limits: EnvironmentLimits, graph_mode: bool,
                 observations_space=("ingress_traffic", "node_load")):
        self.simulator = simulator
        self.env_limits = env_limits
        self.graph_mode = graph_mode
        self.observations_space = list(observations_space)
        self.sfc_dict = {}
        self.node_map = {}
        self.sfc_map = {}
        self.sf_map = {}
        self._edge_index = None

    def init(self, seed) -> Tuple[object, SimulatorState]:
        state = self.simulator.init(seed)
        self.node_map = {node["id"]: i for i, node in enumerate(state.network["nodes"])}
        self.sfc_dict = state.sfcs
        self.sfc_map = {sfc: i for i, sfc in enumerate(state.sfcs)}
        self.sf_map = {sf: i for i, sf in enumerate(state.service_functions)}
        self._edge_index = None
        return (self._parse_state_as_graph(state) if self.graph_mode else self._parse_state(state)), state

    def add_placement_recursive(self, source_node, sf_id, sfc, schedule, placement):
        sf = self.sfc_dict[sfc][sf_id]
        for target, w in schedule[source_node][sfc][sf].items():
            if w > 0:
                placement[target].add(sf)
                if sf_id + 1 < len(self.sfc_dict[sfc]):
                    self.add_placement_recursive(target, sf_id + 1, sfc, schedule, placement)

    def action_to_simulator_action(self, action_array: np.ndarray) -> SimulatorAction:
        lim = self.env_limits
        n = len(self.node_map)
        mask = lim.action_mask(n)
        sched = np.asarray(action_array)[mask == 1].reshape(n, lim.MAX_SF_CHAIN_COUNT,
                                                           lim.MAX_SERVICE_FUNCTION_COUNT, n)
        scheduling = {v: {sfc: {sf: {} for sf in self.sf_map} for sfc in self.sfc_map} for v in self.node_map}
        placement = {v: set() for v in self.node_map}
        for src, si in self.node_map.items():
            for sfc, ci in self.sfc_map.items():
                for sf, fi in self.sf_map.items():
                    row = scheduling[src][sfc][sf]
                    for dst, di in self.node_map.items():
                        row[dst] = sched[si, ci, fi, di]
        for sfc in self.sfc_map:
            for ing in self.simulator.get_active_ingress_nodes():
                self.add_placement_recursive(ing, 0, sfc, scheduling, placement)
        return SimulatorAction(placement, scheduling)

    def apply(self, action_array: np.ndarray) -> Tuple[object, SimulatorState]:
        state = self.simulator.apply(self.action_to_simulator_action(action_array))
        return (self._parse_state_as_graph(state) if self.graph_mode else self._parse_state(state)), state

    def _parse_state(self, state: SimulatorState) -> np.ndarray:
        feats = node_features(state, self.node_map, self.observations_space)
        flat = feats.T.reshape(-1).astype(np.float64)  # feature-major concatenation as in the reference
        if getattr(self.simulator, "test_mode", False) and hasattr(self.simulator, "writer"):
            self.simulator.writer.write_rl_state([self.simulator.episode, self.simulator.env.now] + flat.tolist())
        return flat

    def _graph_edge_index(self) -> torch.Tensor:
        if self._edge_index is None:
            g = getattr(self.simulator, "network", None)
            if g is not None:
                src, dst = [], []
                for u in g.nodes:
                    for v in g.adj[u]:
                        src.append(self.node_map[u])
                        dst.append(self.node_map[v])
                self._edge_index = torch.tensor([src, dst], dtype=torch.long)
            else:
                self._edge_index = torch.zeros((2, 0), dtype=torch.long)
        return self._edge_index

    def _parse_state_as_graph(self, state: SimulatorState) -> GraphObs:
        feats = node_features(state, self.node_map, self.observations_space)
        n = len(state.network["nodes"])
        mask = torch.from_numpy(self.env_limits.action_mask(n)).view(1, -1)
        return GraphObs(torch.from_numpy(feats), self._graph_edge_index().clone(), mask)

    # flat-mode node shuffling (reference simulator_wrapper.py:310-369) ---------------------------
    def permute_node_order(self, state, perm=None):
        n = len(self.node_map)
        if perm is None:
            perm = np.random.permutation(n)
        k = len(state) // n
        assert len(perm) == n and len(state) == k * n
        return np.concatenate([np.asarray(state)[f * n:(f + 1) * n][perm] for f in range(k)]), perm

    @staticmethod
    def reverse_permutation(permutation):
        inverse = [0] * len(permutation)
        for idx, pos in enumerate(permutation):
            inverse[pos] = idx
        return inverse

    def reverse_node_permutation(self, action, node_perm):
        n = len(self.node_map)
        rev = self.reverse_permutation(node_perm)
        per_src = len(self.sfc_map) * len(self.sf_map)
        a = np.asarray(action).reshape(n, per_src, n)
        return a[rev][:, :, rev].reshape(-1)
