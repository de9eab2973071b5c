"""Optimizer-state rewiring after pruning (reference: torchpruner/pruner/opt_pruner.py:4-19).

The reference handles SGD momentum only, looks at ``param_groups[0]`` only, and finds the
buffer through ``optimizer.state_dict()["state"][id(p)]`` — a torch<=1.4 key scheme that
raises KeyError on modern torch (state_dict is keyed by integer index). This version reads
``optimizer.state[param]`` directly, covers every param group, and slices every tensor state
with the parameter's rank (SGD ``momentum_buffer``, Adam/AdamW ``exp_avg``/``exp_avg_sq``/
``max_exp_avg_sq``, RMSprop ``square_avg``/``grad_avg``, Adagrad ``sum``, ...).
"""
from __future__ import annotations

import torch

from .. import ops


class OptimizerPruner:
    @staticmethod
    def _owns(optimizer, param) -> bool:
        return any(p is param for g in optimizer.param_groups for p in g["params"])

    @staticmethod
    def state_tensors(optimizer, param):
        """``[(key, tensor)]`` optimizer states that must be sliced together with ``param``
        (called *before* the parameter itself is sliced)."""
        if optimizer is None or not OptimizerPruner._owns(optimizer, param):
            return []
        st = optimizer.state.get(param, {})
        out = []
        for k, v in st.items():
            if isinstance(v, torch.Tensor) and v.dim() == param.dim() and tuple(v.shape) == tuple(param.shape):
                out.append((k, v))
        return out

    @staticmethod
    def prune(optimizer, param, axis, keep_indices, device=None):
        """Slice the states of an already-pruned ``param`` (reference-compatible entry point)."""
        if optimizer is None or not OptimizerPruner._owns(optimizer, param):
            return
        st = optimizer.state.get(param, {})
        keep = torch.as_tensor(keep_indices, dtype=torch.long)
        items = [(k, v) for k, v in st.items()
                 if isinstance(v, torch.Tensor) and v.dim() == param.dim() and tuple(v.shape) != tuple(param.shape)
                 and v.shape[axis] > keep.numel()]
        if not items:
            return
        outs = ops.gather_multi([v for _, v in items], [axis] * len(items), keep.to(items[0][1].device))
        for (k, _), new in zip(items, outs):
            st[k] = new
