"""Tracing hooks (SURVEY.md §5 "Tracing / profiling").

``trace_range(name)`` emits a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm) when
``TORCHPRUNER_TRACE=1`` so rocprofv3 ``--marker-trace``/torch.profiler timelines show the
engine's phases (forward, backward, fold, collectives); otherwise it costs nothing.
``profile_steps`` wraps a callable in ``torch.profiler`` and returns the key-averages table.
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = os.environ.get("TORCHPRUNER_TRACE", "0") == "1"


def set_tracing(enabled: bool) -> None:
    """Turn the roctx ranges on/off at run time (default: ``TORCHPRUNER_TRACE=1``)."""
    global _ENABLED
    _ENABLED = bool(enabled)


def tracing() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str):
    """A roctx range named ``name`` (rocprofv3 --marker-trace) while tracing is on. Ranges used
    by the package: ``tp.run/<Metric>``, ``tp.forward``, ``tp.backward``, ``tp.fold``,
    ``tp.collective``, ``tp.shapley.prefixes``, ``tp.prune``."""
    if not _ENABLED or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def range_push(name: str) -> bool:
    """Open a roctx range when tracing (pair with :func:`range_pop` if it returned True)."""
    if not _ENABLED or not torch.cuda.is_available():
        return False
    torch.cuda.nvtx.range_push(name)
    return True


def range_pop(opened: bool) -> None:
    if opened:
        torch.cuda.nvtx.range_pop()


def profile_steps(fn, steps: int = 3, row_limit: int = 25, sort_by: str = "cuda_time_total"):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        for _ in range(steps):
            fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    return prof.key_averages().table(sort_by=sort_by, row_limit=row_limit)
