"""Per-topology message-passing tables for batched GNN evaluation.

The reference collates PyG ``Data`` objects into a ``Batch`` every update (``buffer.py:64-84``).
Here every topology used in a run is registered once; a batch of graphs is then just
``(x [B, n_pad, F], topo_id [B])``.  For each topology the table holds the GATv2 message list
in PyG order — the bidirectional edges of ``from_networkx`` followed by one self loop per node
(``GATv2Conv(add_self_loops=True)``) — padded to ``M`` messages, plus in-degrees and the node
mask used by ``global_mean_pool``.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from gsc_amd.coordsim.reader import Topology


class GraphSet:
    def __init__(self, topologies: Sequence[Topology], n_pad: int, device="cpu"):
        self.topologies = list(topologies)
        self.n_pad = int(n_pad)
        T = len(self.topologies)
        msgs = []
        for t in self.topologies:
            ei = t.edge_index()
            keep = ei[0] != ei[1]
            ei = ei[:, keep]
            loops = np.arange(t.n, dtype=np.int64)
            msgs.append((np.concatenate([ei[0], loops]), np.concatenate([ei[1], loops])))
        self.M = max(len(s) for s, _ in msgs)
        # every (source, target) pair at most once: the MFMA kernels scatter attention weights into a
        # dense [target][source] matrix (gsc_amd/ops/gnn.py falls back to other kernels otherwise)
        self.unique_messages = all(len(set(zip(s.tolist(), d.tolist()))) == len(s) for s, d in msgs)
        src = np.zeros((T, self.M), np.int64)
        dst = np.zeros((T, self.M), np.int64)
        valid = np.zeros((T, self.M), bool)
        deg = np.ones((T, self.n_pad), np.float32)
        node_mask = np.zeros((T, self.n_pad), np.float32)
        n_nodes = np.zeros(T, np.float32)
        for i, (t, (s, d)) in enumerate(zip(self.topologies, msgs)):
            m = len(s)
            src[i, :m], dst[i, :m], valid[i, :m] = s, d, True
            cnt = np.bincount(d, minlength=self.n_pad).astype(np.float32)
            deg[i] = np.maximum(cnt, 1.0)
            node_mask[i, :t.n] = 1.0
            n_nodes[i] = t.n
        dev = torch.device(device)
        self.src = torch.from_numpy(src).to(dev)
        self.dst = torch.from_numpy(dst).to(dev)
        self.valid = torch.from_numpy(valid).to(dev)
        self.deg = torch.from_numpy(deg).to(dev)
        self.node_mask = torch.from_numpy(node_mask).to(dev)
        self.n_nodes = torch.from_numpy(n_nodes).to(dev)
        # int32/int16 copies for the HIP kernels
        self.src_i32 = self.src.to(torch.int32)
        self.dst_i32 = self.dst.to(torch.int32)
        self.num_msgs = torch.tensor([len(s) for s, _ in msgs], dtype=torch.int32, device=dev)
        # CSR views of the message list (stable in message order) for the fused HIP kernels:
        # messages into each node (softmax + aggregation) and out of each node (d x_l).
        self.max_nodes = max(t.n for t in self.topologies)
        in_ptr = np.zeros((T, self.n_pad + 1), np.int32)
        out_ptr = np.zeros((T, self.n_pad + 1), np.int32)
        in_msg = np.zeros((T, self.M), np.int32)
        out_msg = np.zeros((T, self.M), np.int32)
        for i, (s, d) in enumerate(msgs):
            for key, ptr, lst in ((d, in_ptr, in_msg), (s, out_ptr, out_msg)):
                order = np.argsort(key, kind="stable")
                lst[i, :len(order)] = order
                cnt = np.bincount(key, minlength=self.n_pad)
                ptr[i, 1:] = np.cumsum(cnt)
        # CSR-ordered message arrays (fused + layer-wise kernels): messages sorted by target node keep
        # their source/target directly, and the source-sorted view stores positions in that order.
        in_src = np.zeros((T, self.M), np.int32)
        in_dst = np.zeros((T, self.M), np.int32)
        out_q = np.zeros((T, self.M), np.int32)
        out_dst = np.zeros((T, self.M), np.int32)
        for i, (s, d) in enumerate(msgs):
            m = len(s)
            pos = np.empty(m, np.int64)
            pos[in_msg[i, :m]] = np.arange(m)
            in_src[i, :m] = s[in_msg[i, :m]]
            in_dst[i, :m] = d[in_msg[i, :m]]
            out_q[i, :m] = pos[out_msg[i, :m]]
            out_dst[i, :m] = d[out_msg[i, :m]]
        self.in_src = torch.from_numpy(in_src).to(dev)
        self.in_dst = torch.from_numpy(in_dst).to(dev)
        self.out_q = torch.from_numpy(out_q).to(dev)
        self.out_dst = torch.from_numpy(out_dst).to(dev)
        # lane -> node maps of the large-graph kernels (csrc/ops/gnn_lg.hip): nodes by in-degree (row 0) and by
        # out-degree (row 1), descending (stable; padded nodes last), so each wave's 32 nodes have similar
        # degrees and the per-node message loops waste few lane-iterations on shorter segments
        order = np.zeros((T, 2, self.n_pad), np.int32)
        for i in range(T):
            for r, ptr in enumerate((in_ptr, out_ptr)):
                d = np.diff(ptr[i])
                order[i, r] = np.argsort(-d, kind="stable")
        self.deg_order = torch.from_numpy(order).to(dev)
        self.in_ptr = torch.from_numpy(in_ptr).to(dev)
        self.in_msg = torch.from_numpy(in_msg).to(dev)
        self.out_ptr = torch.from_numpy(out_ptr).to(dev)
        self.out_msg = torch.from_numpy(out_msg).to(dev)
        self.n_nodes_i32 = self.n_nodes.to(torch.int32)
        # one-hot message matrices of the MFMA backward (csrc/ops/gnn_mf.hip, gnn_mt.hip), bf16
        # [T, 32 * tiles, MP] (one 32-node tile up to 32 nodes, two up to 64): s_dst[t, i, q] = 1 if
        # message q (target-sorted order) ends at node i, s_src likewise for its source; dX_r = s_dst G
        # and dX_l = s_src G are then matrix-core products
        self.mf_mp = ((self.M + 15) // 16) * 16
        rows = 32 * max(1, -(-self.max_nodes // 32)) if self.max_nodes <= 64 else 32
        s_dst = np.zeros((T, rows, self.mf_mp), np.float32)
        s_src = np.zeros((T, rows, self.mf_mp), np.float32)
        if self.max_nodes <= 64:
            for i, (s, _) in enumerate(msgs):
                q = np.arange(len(s))
                s_dst[i, in_dst[i, :len(s)], q] = 1.0
                s_src[i, in_src[i, :len(s)], q] = 1.0
        self.s_dst = torch.from_numpy(s_dst).to(dev, torch.bfloat16)
        self.s_src = torch.from_numpy(s_src).to(dev, torch.bfloat16)

    @property
    def num_topologies(self) -> int:
        return len(self.topologies)

    def to(self, device) -> "GraphSet":
        return GraphSet(self.topologies, self.n_pad, device)

    def action_masks(self, C: int, F: int) -> torch.Tensor:
        """``[T, n_pad*C*F*n_pad]`` masks with ones on each topology's real ``[:n, :, :, :n]`` block."""
        P = self.n_pad
        out = torch.zeros((self.num_topologies, P, C, F, P), dtype=torch.float32)
        for i, t in enumerate(self.topologies):
            out[i, :t.n, :, :, :t.n] = 1
        return out.reshape(self.num_topologies, -1).to(self.src.device)
