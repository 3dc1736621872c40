"""Phase tracing: roctx ranges + an in-process phase timer / steps-per-second counter.

The reference has no profiler hooks: only ``ExperimentResult.runtime_*``,
``Metrics.running_time``, ``runtimes.csv`` and an unreachable ``charts/SPS`` tag.

* ``GSC_TRACE=1`` wraps every :func:`trace_range` in a roctx range (``torch.cuda.nvtx`` is the
  roctx binding on ROCm builds), so ``rocprofv3 --marker-trace`` shows act / explore / sim /
  replay / learn / all-reduce phases next to the kernels.
* ``GSC_TRACE_SYNC=1`` additionally synchronises the device at range boundaries and accumulates
  wall time per phase in :data:`PHASES` (exact attribution at the cost of overlap — for analysis
  runs only).
* :class:`SPSCounter` is the working equivalent of the reference's ``charts/SPS``.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict

import torch

_TRACE = os.environ.get("GSC_TRACE", "0") not in ("", "0")
_SYNC = os.environ.get("GSC_TRACE_SYNC", "0") not in ("", "0")
PHASES: Dict[str, float] = defaultdict(float)
COUNTS: Dict[str, int] = defaultdict(int)


def enabled() -> bool:
    return _TRACE or _SYNC


def set_tracing(on: bool, sync: bool = False) -> None:
    global _TRACE, _SYNC
    _TRACE, _SYNC = bool(on), bool(sync)


def _marker_ok() -> bool:
    return torch.cuda.is_available() and hasattr(torch.cuda, "nvtx")


@contextlib.contextmanager
def trace_range(name: str):
    if not (_TRACE or _SYNC):
        yield
        return
    mark = _TRACE and _marker_ok()
    if _SYNC and torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mark:
        torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        if mark:
            torch.cuda.nvtx.range_pop()
        if _SYNC and torch.cuda.is_available():
            torch.cuda.synchronize()
        PHASES[name] += time.perf_counter() - t0
        COUNTS[name] += 1


def phase_report(reset: bool = True) -> Dict[str, float]:
    """Mean milliseconds per call of every traced phase (meaningful with ``GSC_TRACE_SYNC=1``)."""
    out = {f"time/{k}_ms": 1e3 * v / max(COUNTS[k], 1) for k, v in PHASES.items()}
    if reset:
        PHASES.clear()
        COUNTS.clear()
    return out


class SPSCounter:
    """Environment steps per second since the last :meth:`rate` call."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self.n = 0

    def add(self, steps: int) -> None:
        self.n += int(steps)

    def rate(self, reset: bool = True) -> float:
        dt = time.perf_counter() - self.t0
        r = self.n / dt if dt > 0 else 0.0
        if reset:
            self.t0, self.n = time.perf_counter(), 0
        return r
