"""Tracing hooks.

* ``phase_range(name)``: a roctx range (``torch.cuda.nvtx`` is backed by roctx on ROCm) around a step
  phase, visible in ``rocprofv3 --marker-trace`` / Perfetto timelines; free when no GPU is present.
* ``StepTimer``: host-side step-time breakdown (device-synchronised), for the trainer/bench logs.
* ``torch.profiler`` traces are taken by the trainer with ``--profile_steps N``; per-kernel device time
  comes from ``rocprofv3 --kernel-trace --stats`` (see tools/prof_summary.py and profiles/).
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch

_ROCTX = torch.cuda.is_available()


@contextlib.contextmanager
def phase_range(name: str):
    if _ROCTX:
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    """Accumulates wall time per named phase (synchronising the device at phase boundaries)."""

    def __init__(self, sync: bool = True):
        self.sync = sync and torch.cuda.is_available()
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        with phase_range(name):
            yield
        if self.sync:
            torch.cuda.synchronize()
        self.total[name] += time.perf_counter() - t0
        self.count[name] += 1

    def report(self) -> str:
        return "  ".join(f"{k}: {1e3 * v / max(self.count[k], 1):.3f} ms" for k, v in self.total.items())
