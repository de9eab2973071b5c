"""Host -> device batch prefetching on a side HIP stream (copy / compute overlap).

The reference feeds attribution passes from CPU DataLoaders and copies every batch with a
blocking ``.to(device)`` right before using it (attributions.py:48-50,64-66), so the H2D copy
and the kernels of the previous batch never overlap. ``prefetch_to_device`` keeps ``depth``
batches in flight: batch i+1 is pinned and copied on a dedicated copy stream while batch i is
being consumed on the compute stream; the consumer waits on a per-batch event only, and the
tensors are recorded on the compute stream so the caching allocator never recycles them early.
"""
from __future__ import annotations

from collections import deque
from typing import Iterable, Iterator

import torch


def _pinned(t):
    if isinstance(t, torch.Tensor) and not t.is_cuda and not t.is_pinned():
        return t.pin_memory()
    return t


def _copy(t, device):
    return t.to(device, non_blocking=True) if isinstance(t, torch.Tensor) else t


def prefetch_to_device(items: Iterable[tuple], device, depth: int = 2) -> Iterator[tuple]:
    """Yield the tuples of ``items`` with every tensor moved to ``device``; copies of the next
    ``depth`` tuples run ahead on a side stream. Non-CUDA devices pass through with a plain
    copy; tuples already on the device cost nothing extra."""
    device = torch.device(device)
    if device.type != "cuda":
        for item in items:
            yield tuple(_copy(t, device) for t in item)
        return
    copy_stream = torch.cuda.Stream(device)
    pending = deque()
    it = iter(items)

    def issue():
        try:
            item = next(it)
        except StopIteration:
            return False
        with torch.cuda.stream(copy_stream):
            moved = tuple(_copy(_pinned(t), device) for t in item)
            ev = torch.cuda.Event()
            ev.record(copy_stream)
        pending.append((moved, ev))
        return True

    for _ in range(max(1, depth)):
        if not issue():
            break
    compute = torch.cuda.current_stream(device)
    while pending:
        moved, ev = pending.popleft()
        compute.wait_event(ev)
        for t in moved:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(compute)
        issue()
        yield moved
