"""Graph observation containers (replaces PyG ``Data``/``Batch`` used by the reference).

``GraphObs`` holds one graph (``x [n, F]``, ``edge_index [2, 2E]``, ``mask [1, A]``).
``GraphBatch`` is the collated form (``x [sum n, F]``, offset ``edge_index``,
``batch`` vector, ``mask [B, A]``) — the same layout PyG's
``Batch.from_data_list`` produces (reference ``buffer.py:64-87``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch


@dataclass
class GraphObs:
    x: torch.Tensor
    edge_index: torch.Tensor
    mask: torch.Tensor

    @property
    def num_nodes(self) -> int:
        return int(self.x.shape[0])

    def clone(self) -> "GraphObs":
        return GraphObs(self.x.clone(), self.edge_index.clone(), self.mask.clone())

    def to(self, device) -> "GraphObs":
        return GraphObs(self.x.to(device), self.edge_index.to(device), self.mask.to(device))

    def batch(self) -> "GraphBatch":
        return GraphBatch.from_list([self])


@dataclass
class GraphBatch:
    x: torch.Tensor
    edge_index: torch.Tensor
    batch: torch.Tensor
    mask: torch.Tensor
    num_graphs: int
    nodes_per_graph: Optional[int] = None  # set when every graph has the same node count (dense fast path)

    @staticmethod
    def from_list(items: List[GraphObs]) -> "GraphBatch":
        xs, eis, bs = [], [], []
        off = 0
        sizes = set()
        for i, g in enumerate(items):
            n = g.num_nodes
            sizes.add(n)
            xs.append(g.x)
            eis.append(g.edge_index + off)
            bs.append(torch.full((n,), i, dtype=torch.long, device=g.x.device))
            off += n
        mask = torch.cat([g.mask.reshape(1, -1) for g in items], 0)
        return GraphBatch(torch.cat(xs, 0), torch.cat(eis, 1), torch.cat(bs, 0), mask, len(items),
                          sizes.pop() if len(sizes) == 1 else None)

    def to(self, device) -> "GraphBatch":
        return GraphBatch(self.x.to(device), self.edge_index.to(device), self.batch.to(device),
                          self.mask.to(device), self.num_graphs, self.nodes_per_graph)
