"""Checkpoint / resume (SURVEY.md §5 "Checkpoint / resume").

Pruned models: the reference's pruned ``state_dict`` keeps every key and only the tensor
shapes shrink (pruner.py:94-115), so reloading needs a model with the pruned widths. Here
:func:`save_pruned` stores the state_dict together with a manifest of per-module widths and
Dropout rates, and :func:`load_pruned` shrinks a freshly constructed (unpruned) model to
the saved shapes — parameters, buffers and module metadata — before ``load_state_dict``.
Files load with ``torch.load(..., weights_only=True)`` (tensors + plain containers only).

Attribution runs: :class:`AttributionCheckpoint` persists the device accumulators (fp64
score sums / per-sample slabs) plus the set of processed global batch indices, so a run
interrupted by a failure resumes at the next unprocessed batch (e.g. under torchrun's
elastic restarts).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch
import torch.nn as nn
from torch.nn.modules.batchnorm import _BatchNorm
from torch.nn.modules.conv import _ConvNd, _ConvTransposeNd
from torch.nn.modules.dropout import _DropoutNd


def pruned_manifest(model: nn.Module) -> dict:
    mods = {}
    for name, m in model.named_modules():
        if isinstance(m, _ConvNd):
            mods[name] = {"type": "conv", "in": m.in_channels, "out": m.out_channels}
        elif isinstance(m, nn.Linear):
            mods[name] = {"type": "linear", "in": m.in_features, "out": m.out_features}
        elif isinstance(m, _BatchNorm):
            mods[name] = {"type": "bn", "num_features": m.num_features}
        elif isinstance(m, _DropoutNd):
            mods[name] = {"type": "dropout", "p": float(m.p)}
    return {"format": "torchpruner_amd.pruned/1", "modules": mods}


def save_pruned(model: nn.Module, path: str, optimizer: Optional[torch.optim.Optimizer] = None,
                extra: Optional[dict] = None) -> None:
    payload = {"state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
               "manifest": json.dumps(pruned_manifest(model))}
    if optimizer is not None:
        payload["optimizer"] = optimizer.state_dict()
    if extra:
        payload["extra"] = json.dumps(extra)
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def shrink_to_state_dict(model: nn.Module, state_dict: dict, manifest: Optional[dict] = None) -> nn.Module:
    """Resize every parameter/buffer of ``model`` to the shapes in ``state_dict`` (Parameter
    identity preserved) and update module metadata so the model can load it."""
    modules = dict(model.named_modules())
    for key, t in state_dict.items():
        mod_name, _, attr = key.rpartition(".")
        m = modules.get(mod_name)
        if m is None:
            continue
        cur = getattr(m, attr, None)
        if isinstance(cur, torch.Tensor) and tuple(cur.shape) != tuple(t.shape):
            cur.data = torch.empty(t.shape, dtype=cur.dtype, device=cur.device)
    for name, m in modules.items():
        if isinstance(m, _ConvNd):
            w = m.weight
            transposed = isinstance(m, _ConvTransposeNd)
            m.out_channels = w.shape[1] * m.groups if transposed else w.shape[0]
            m.in_channels = w.shape[0] if transposed else w.shape[1] * m.groups
        elif isinstance(m, nn.Linear):
            m.out_features, m.in_features = m.weight.shape
        elif isinstance(m, _BatchNorm):
            ref = m.running_mean if m.running_mean is not None else m.weight
            if ref is not None:
                m.num_features = ref.shape[0]
    if manifest:
        for name, info in manifest.get("modules", {}).items():
            m = modules.get(name)
            if info.get("type") == "dropout" and isinstance(m, _DropoutNd):
                m.p = info["p"]
    return model


def load_pruned(model: nn.Module, path_or_payload, strict: bool = True, optimizer=None) -> nn.Module:
    payload = path_or_payload
    if isinstance(path_or_payload, (str, os.PathLike)):
        payload = torch.load(path_or_payload, map_location="cpu", weights_only=True)
    sd = payload["state_dict"] if "state_dict" in payload else payload
    manifest = json.loads(payload["manifest"]) if isinstance(payload, dict) and "manifest" in payload else None
    shrink_to_state_dict(model, sd, manifest)
    model.load_state_dict(sd, strict=strict)
    if optimizer is not None and "optimizer" in payload:
        optimizer.load_state_dict(payload["optimizer"])
    return model


class AttributionCheckpoint:
    """Persist/restore the accumulators of an attribution run every ``every`` batches."""

    def __init__(self, path: str, key: str, every: int = 50):
        self.path = path
        self.key = key
        self.every = max(1, int(every))
        self.done: set[int] = set()
        self._since = 0

    def restore(self, accs) -> set:
        if not os.path.exists(self.path):
            return set()
        st = torch.load(self.path, map_location="cpu", weights_only=True)
        if st.get("key") != self.key:
            return set()
        for a, s in zip(accs, st["accs"]):
            dev = a.device
            if s.get("sum") is not None:
                a.sum = s["sum"].to(dev)
            a.count = int(s["count"])
            a.width = s.get("width")
            a.slabs = [(int(i), t.to(dev)) for i, t in s.get("slabs", [])]
            if s.get("dtype") == "float32":
                a.dtype = torch.float32
        self.done = set(int(i) for i in st["done"])
        return self.done

    def step(self, accs, batch_index: int, force: bool = False):
        self.done.add(int(batch_index))
        self._since += 1
        if force or self._since >= self.every:
            self.save(accs)

    def save(self, accs):
        self._since = 0
        st = {"key": self.key, "done": sorted(self.done), "accs": []}
        for a in accs:
            st["accs"].append({"sum": a.sum.cpu() if a.sum is not None else None, "count": a.count,
                               "width": a.width,
                               "slabs": [(i, t.cpu()) for i, t in a.slabs],
                               "dtype": "float32" if a.dtype in (None, torch.float32) else "float64"})
        tmp = self.path + ".tmp"
        torch.save(st, tmp)
        os.replace(tmp, self.path)
