"""Data parallelism (RCCL over xGMI on GPU, gloo on CPU)."""
from .dist import DistInfo, allreduce_sum_, barrier, broadcast_tensors, init_distributed, shutdown
