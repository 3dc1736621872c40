"""Fixed-size action/observation spaces (reference: ``src/rlsp/envs/environment_limits.py``).

Action layout is ``(src_node, sfc, sf, dst_node)`` flattened, padded to
``MAX_NODE_COUNT`` nodes; ``MAX_SERVICE_FUNCTION_COUNT`` is the longest chain.
"""
import numpy as np

from .spaces import Box, Dict


class EnvironmentLimits:
    def __init__(self, num_nodes: int, sfc_list, node_obs_space_len: int, link_obs_space_len: int,
                 num_edges: int, graph_mode: bool = False):
        self.MAX_NODE_COUNT = int(num_nodes)
        self.MAX_SF_CHAIN_COUNT = len(sfc_list)
        self.observation_space_len = node_obs_space_len
        self.link_obs_space_len = link_obs_space_len
        self.graph_mode = graph_mode
        self.num_edges = int(num_edges)
        self.MAX_SERVICE_FUNCTION_COUNT = max((len(v) for v in sfc_list.values()), default=0)

    @property
    def node_load_shape(self):
        return (self.MAX_NODE_COUNT,)

    @property
    def scheduling_shape(self):
        return (self.MAX_NODE_COUNT, self.MAX_SF_CHAIN_COUNT, self.MAX_SERVICE_FUNCTION_COUNT, self.MAX_NODE_COUNT)

    @property
    def action_dim(self) -> int:
        return int(np.prod(self.scheduling_shape))

    @property
    def action_space(self):
        return Box(low=0, high=1, shape=(self.action_dim,))

    @property
    def observation_space(self):
        if not self.graph_mode:
            return Box(0, 1, shape=(self.observation_space_len * self.MAX_NODE_COUNT,), dtype=np.float32)
        return Dict({
            "nodes": Box(0, 1, shape=(self.MAX_NODE_COUNT, self.observation_space_len), dtype=np.float32),
            "adj": Box(0, 1000, shape=(2, 2 * self.num_edges), dtype=np.int64),
        })

    def create_filled_node_load_array(self, default=0.0):
        return np.full(self.node_load_shape, default, dtype=float)

    def action_mask(self, n: int) -> np.ndarray:
        """1 on the real ``[:n, :, :, :n]`` block of the padded action."""
        m = np.zeros(self.scheduling_shape, dtype=np.float32)
        m[:n, :, :, :n] = 1
        return m.reshape(-1)
