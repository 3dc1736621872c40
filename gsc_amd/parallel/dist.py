"""Data parallelism over RCCL/xGMI (one process per GPU) with a CPU/gloo path for tests.

Environment shards are disjoint per rank (each rank steps its own E envs and keeps its own replay
ring); the actor and critic are replicated: parameters (and targets) are broadcast from rank 0 at
start / resume and each network's flat gradient buffer is all-reduced once per update (a single
contiguous bucket — ~4.5 MB at Abilene scale, latency-bound on xGMI, so one collective beats any
bucketing), summed and rescaled inside the fused Adam kernel.  Scalar metrics are summed with one
small all-reduce.  The reference is single-process: this layer is
new capability.

``GSC_DIST_FORCE=1`` with a single process builds a world-size-1 process group (RCCL on a GPU, gloo on the
CPU) and routes every collective through it: the data-parallel code path (the gradient all-reduces captured
in the update graph, or the fallback's eager collectives between five per-stage graphs, ZeRO-1
reduce-scatter / all-gather, replica checks) then runs on one GPU,
bit-identical to the process-local learner.  ``GSC_DP_GRAD_BF16=1`` all-reduces gradients in bf16 (half
the xGMI bytes; fp32 master weights and Adam are unchanged, see ``GradReduce``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    forced: bool = False   # GSC_DIST_FORCE=1: a world-size-1 process group, collectives issued anyway

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.forced

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(device_type: str = "cuda", timeout_s: int = 600) -> DistInfo:
    """Initialise the process group from torchrun's env vars (no-op when WORLD_SIZE is unset/1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    forced = world <= 1 and os.environ.get("GSC_DIST_FORCE", "0") == "1"
    if world <= 1 and not forced:
        return DistInfo(0, 1, local, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # GSC_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several ranks on one GPU
    # (RCCL refuses two ranks per device); the default on GPUs is RCCL ("nccl")
    backend = os.environ.get("GSC_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if device_type == "cuda":
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        # RCCL async error handling: a hung peer surfaces as an exception instead of a silent hang
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if forced:  # one process: an in-memory store, no rendezvous
            kw.update(store=dist.HashStore(), rank=0, world_size=1)
        if device_type == "cuda" and backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        try:
            dist.init_process_group(**kw)
        except TypeError:  # older torch without device_id
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    return DistInfo(0 if forced else rank, 1 if forced else world, local, backend, forced)


def shutdown() -> None:
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _active() -> bool:
    """A process group exists (world size > 1, or the forced world-size-1 group)."""
    return dist.is_available() and dist.is_initialized()


def broadcast_tensors(tensors: List[torch.Tensor], src: int = 0) -> None:
    if _active():
        for t in tensors:
            dist.broadcast(t, src)


def allreduce_sum_(t: torch.Tensor, async_op: bool = False):
    if _active():
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
    return None


def barrier() -> None:
    if _active():
        dist.barrier()


def allreduce_max_scalar(x: float, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if _active():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sync_string(s: str, src: int = 0) -> str:
    """Rank ``src``'s value of a short string on every rank (run ids, seeds)."""
    if not (dist.is_available() and dist.is_initialized()):
        return s
    obj = [s]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


class GradReduce:
    """Sum-all-reduce of a flat gradient slice, optionally in bf16 (``GSC_DP_GRAD_BF16=1``).

    bf16 mode: the slice is rounded into a bf16 staging buffer on the compute stream, the collective sums
    the staging buffer (half the bytes on xGMI: the config-5 gradient is 0.92 GB in fp32), and ``wait()``
    widens the sum back into the fp32 gradient on the compute stream, where the fused Adam kernel
    (fp32 master weights and moments) reads it.  The rounding error is one bf16 ulp per rank's
    contribution plus the collective's bf16 partial sums; ``tests/test_distributed.py`` bounds its effect
    on an update against the fp32 reduction."""

    def __init__(self, grad: torch.Tensor, staging: Optional[torch.Tensor]):
        self.grad, self.staging = grad, staging
        if staging is not None:
            staging.copy_(grad)
            self.work = dist.all_reduce(staging, op=dist.ReduceOp.SUM, async_op=True)
        else:
            self.work = dist.all_reduce(grad, op=dist.ReduceOp.SUM, async_op=True)

    def wait(self) -> None:
        if self.work is not None:
            self.work.wait()
        if self.staging is not None:
            self.grad.copy_(self.staging)
