"""Sharded optimizer state for data parallelism (ZeRO stage 1) over RCCL / gloo.

With the plain data-parallel path every rank all-reduces each network's flat gradient and runs the full
fused Adam + Polyak pass.  At config-5 scale (200-node topologies, 3 SFCs: A = 360,000, ~230 M actor +
critic parameters) that pass reads/writes ~36 B per parameter on every rank (1.76 ms/step at 5.2 TB/s,
``profiles/bench_1gpu_syn200_kernels.txt``) and every rank holds both Adam moments.  Sharded:

    reduce-scatter(grad bucket)  ->  rank r owns 1/W of the summed gradient
    guard: non-finite check of the shard, ranks agree (all-reduce MAX of one int)
    Adam on the shard only (moments of 1/W of the parameters)
    all-gather(parameters)       ->  every rank holds the updated fp32 parameters again
    Polyak target update + bf16 shadows over the whole buffer (bit-identical on every rank: the same inputs)

Communication per update equals the all-reduce's (a ring all-reduce is a reduce-scatter followed by an
all-gather); the optimizer pass shrinks to 1/W plus one elementwise Polyak/shadow pass, and the moments
to 1/W of the memory.  Buckets follow the flat buffer's runs: the actor's embedder block and its MLP block
are separate buckets (the MLP bucket's reduce-scatter overlaps the embedder backward, as the all-reduce
does on the unsharded path).  Every bucket is padded to a multiple of 8 W elements inside the flat buffer
(``FlatParams(bucket_align=8 W)``), so all shards are equal and no shard straddles two buckets.

The CPU rehearsal (gloo) issues the same ``reduce_scatter_tensor`` / ``all_gather_into_tensor`` calls as
RCCL does on GPUs, and ``GSC_DIST_FORCE=1`` runs them through a world-size-1 RCCL group on one GPU.  SURVEY §2.8 D1 / §5.8 (new capability: the reference is single-process).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


class ZeroShards:
    """The shard layout of one flat buffer: buckets [lo, hi) (multiples of 8 W), each split into W equal
    contiguous shards; rank r owns shard r of every bucket."""

    def __init__(self, buckets: Sequence[Tuple[int, int]], rank: int, world: int):
        self.rank, self.world = int(rank), int(world)
        self.buckets: List[Tuple[int, int]] = []
        for lo, hi in buckets:
            assert (hi - lo) % (8 * world) == 0 and lo % 8 == 0, "bucket must be a multiple of 8 W elements"
            self.buckets.append((int(lo), int(hi)))
        # offset of each bucket's shard inside the rank's local (concatenated) shard buffers
        self.local_off = []
        off = 0
        for lo, hi in self.buckets:
            self.local_off.append(off)
            off += (hi - lo) // world
        self.local_numel = off

    def shard(self, b: int) -> Tuple[int, int]:
        lo, hi = self.buckets[b]
        c = (hi - lo) // self.world
        return lo + self.rank * c, lo + (self.rank + 1) * c

    def chunk(self, b: int) -> int:
        lo, hi = self.buckets[b]
        return (hi - lo) // self.world


def reduce_scatter_bucket(full: torch.Tensor, lo: int, hi: int, out: torch.Tensor, world: int, rank: int,
                          async_op: bool = False):
    """Sum ``full[lo:hi]`` over ranks; ``out`` receives this rank's contiguous 1/W of the sum (one
    ``reduce_scatter_tensor``: RCCL on GPUs, gloo on the CPU -- the same call, shapes and semantics)."""
    assert out.numel() * world == hi - lo
    return dist.reduce_scatter_tensor(out, full[lo:hi], op=dist.ReduceOp.SUM, async_op=async_op)


def all_gather_bucket(full: torch.Tensor, lo: int, hi: int, world: int, rank: int) -> None:
    """Every rank's shard of ``full[lo:hi]`` to every rank (the own shard is the input; it is copied out
    first because the output buffer contains it)."""
    c = (hi - lo) // world
    dst = full[lo:hi]
    mine = dst[rank * c:(rank + 1) * c].clone()
    dist.all_gather_into_tensor(dst, mine)


def agree_any(flag: torch.Tensor) -> None:
    """flag[0] (int32) = max over ranks (the shards' non-finite flags -> one decision everywhere)."""
    dist.all_reduce(flag[:1], op=dist.ReduceOp.MAX)


def bucket_bounds(flat_numel: int, split: Optional[int]) -> List[Tuple[int, int]]:
    """[0, split) and [split, numel) (split 0 / None: one bucket)."""
    if not split:
        return [(0, flat_numel)]
    return [(0, split), (split, flat_numel)]
