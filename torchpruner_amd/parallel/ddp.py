"""Prune-aware DistributedDataParallel (SURVEY.md §2.6 R6/R7, §2.7 "DDP for finetune").

``torch.nn.parallel.DistributedDataParallel`` sizes its gradient buckets (and, with
``gradient_as_bucket_view``, the ``.grad`` storage) from the parameter shapes at construction.
Structured pruning changes those shapes in place (Pruner keeps Parameter identity), so the
wrapper must be rebuilt after every prune: :class:`PrunableDDP` does that, re-broadcasting
the (already identical, see Pruner's index broadcast R5) parameters from rank 0 (R7).

Gradient all-reduce runs on RCCL over xGMI. xGMI is point-to-point (7 links x ~153 GB/s per
MI355X); RCCL's ring/tree channels are per-link bound, so buckets must be large enough to
amortise the per-collective latency, but the LAST bucket is what stays exposed: it becomes
ready only when the backward ends. Measured inside the native ResNet-50 backward (B=128,
``scripts/probes/ddp_overlap_probe.py``, ``profiles/dist/ddp_bucket_overlap_r6.txt``): 91 of the
97.5 MB of gradients (layers 2-4 + fc) are ready within the first 12 ms of a 25 ms backward, the
stage-1 / stem tail produces the rest over the last 13 ms. With 64 MB buckets the last one holds
32.6 MB (~0.34 ms of 8-rank ring at 200 GB/s bus bandwidth after the backward); with 16 MB it
holds 8 MB (~0.11 ms) in 6 collectives, hence the default ``bucket_cap_mb=16``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn.parallel import DistributedDataParallel as DDP

from . import dist as pdist


class PrunableDDP(nn.Module):
    """Wraps ``module`` in DDP when a multi-rank process group is live (identity otherwise)
    and rebuilds the wrapper on :meth:`rewrap` after pruning."""

    def __init__(self, module: nn.Module, device=None, bucket_cap_mb: float = 16.0, **ddp_kwargs):
        super().__init__()
        self.module = module
        self.device = device
        self.bucket_cap_mb = bucket_cap_mb
        self.ddp_kwargs = ddp_kwargs
        self._ddp = None
        self.rewrap()

    @property
    def distributed(self) -> bool:
        return pdist.get_world_size() > 1

    def rewrap(self):
        """(Re)build the DDP wrapper for the current parameter shapes."""
        self._ddp = None
        if not self.distributed:
            return self
        dev = self.device
        kw = dict(self.ddp_kwargs)
        if dev is not None and torch.device(dev).type == "cuda":
            kw.setdefault("device_ids", [torch.device(dev).index or 0])
        kw.setdefault("broadcast_buffers", True)
        self._ddp = DDP(self.module, bucket_cap_mb=self.bucket_cap_mb, **kw)
        return self

    def forward(self, *args, **kwargs):
        if self._ddp is None:
            return self.module(*args, **kwargs)
        return self._ddp(*args, **kwargs)


def prune_and_rewrap(pruner, wrapper: PrunableDDP, module, indices, cascading_modules):
    """Prune ``module`` (+ cascade) on the unwrapped model, then rebuild the DDP buckets."""
    pruner.prune_model(module, indices, cascading_modules=cascading_modules)
    wrapper.rewrap()


def params_in_sync(model: nn.Module, group=None) -> bool:
    """True when every parameter is bitwise identical across ranks (debug / tests)."""
    if pdist.get_world_size(group) == 1:
        return True
    ok = True
    for p in model.parameters():
        t = p.detach().float().flatten()
        ref = t.clone()
        pdist.broadcast_tensor_(ref, 0, group)
        ok = ok and bool(torch.equal(ref, t))
    flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
    return pdist.all_max_float(float(flag.item()), group) == 0.0  # any rank out of sync -> 1
