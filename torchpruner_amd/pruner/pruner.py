"""On-the-fly structured pruning (reference: torchpruner/pruner/pruner.py:14-185).

Same API as the reference — ``Pruner(model, input_size, device, optimizer=None)`` with
``prune_model`` / ``prune_module`` / ``prune_parameter`` — and the same NaN-probe trick to
discover which input channels of each cascading module depend on the pruned units (this
resolves Flatten and MaxPool automatically, test_pruner.py:83-107).

Differences (deliberate fixes):
* the probe runs in eval mode under ``no_grad`` and restores the train/eval flag, so BatchNorm
  running statistics are not polluted by the random/NaN probe batch;
* every tensor that must shrink with a parameter — the parameter, its ``.grad`` and every
  optimizer state of matching shape (SGD momentum, Adam moments, ...) in *every* param group —
  is sliced by ONE multi-tensor HIP gather launch (ops.gather_multi) on GPU;
* module metadata (``in_features``, ``out_channels``, ``num_features``...) is updated;
* ``_DropoutNd`` (Dropout2d etc.) is accepted; grouped convolutions are rejected explicitly;
  transposed convolutions are pruned on their correct weight axes;
* in a live process group the pruning indices are broadcast from rank 0 (R5) so every
  data-parallel replica prunes identically.
"""
from __future__ import annotations

import contextlib
import logging
import os

import numpy as np
import torch
import torch.nn as nn
from torch.nn.modules.batchnorm import _BatchNorm
from torch.nn.modules.conv import _ConvNd, _ConvTransposeNd
from torch.nn.modules.dropout import _DropoutNd

from .. import ops
from ..utils.profiling import trace_range
from ..parallel import dist as pdist
from .opt_pruner import OptimizerPruner

logger = logging.getLogger("torchpruner")

SUPPORTED_IN_PRUNING_MODULES = [nn.Linear, _ConvNd, _DropoutNd, _BatchNorm]
SUPPORTED_OUT_PRUNING_MODULES = [nn.Linear, _ConvNd]


def _as_index_array(indices) -> np.ndarray:
    if isinstance(indices, torch.Tensor):
        indices = indices.detach().cpu().numpy()
    arr = np.asarray(indices, dtype=np.int64).reshape(-1)
    return np.unique(arr)


class Pruner:
    def __init__(self, model, input_size, device, optimizer=None, group=None, sync_indices=True):
        self.model = model
        self.device = device
        self.input_size = input_size
        self.optimizer = optimizer
        self.group = group
        self.sync_indices = sync_indices
        self._depth = 0  # > 0 inside a public call: nested calls use already-agreed indices

    # ------------------------------------------------------------------ public API
    def prune_model(self, module, indices, cascading_modules=None):
        """Prune output units ``indices`` of ``module`` and cascade into ``cascading_modules``."""
        with trace_range("tp.prune"), self._entry():
            return self._prune_model(module, self._sync(_as_index_array(indices)), cascading_modules)

    def _prune_model(self, module, indices, cascading_modules=None):
        if cascading_modules is None:
            logger.warning("no cascading modules defined")
            cascading_modules = []

        # 1. NaN-probe: nanify the pruned output channels, record NaN input channels downstream.
        # What the probe finds lives in a per-call context, not on the modules (the
        # reference stashes _nan_indices / _activation_len on them, pruner.py:155-167, which is
        # not reentrant: two pruners probing one module would overwrite each other's findings)
        probe = _ProbeRun()
        handles = [module.register_forward_hook(self._nanify_hook(indices))]
        for next_module in cascading_modules:
            handles.append(next_module.register_forward_hook(self._detect_nan_hook(probe)))
        try:
            self._run_forward()
        finally:
            for h in handles:
                h.remove()

        # 2. Prune every cascading module whose input saw NaNs (inputs), then the module (outputs)
        for next_module in cascading_modules:
            idx = probe.nan_indices.get(next_module)
            if idx is not None:
                self._prune_module(next_module, _as_index_array(idx), direction="in",
                                   original_len=probe.activation_len.get(next_module))
        self._prune_module(module, indices, direction="out")

    def prune_module(self, module, indices, direction="out", original_len=None):
        """Prune a module's parameters along its output (``"out"``) or input (``"in"``) units."""
        with self._entry():
            return self._prune_module(module, self._sync(_as_index_array(indices)), direction, original_len)

    def _prune_module(self, module, indices, direction="out", original_len=None):
        assert direction in ["out", "in"], "direction should be 'out' or 'in'"
        if direction == "out":
            assert any(isinstance(module, t) for t in SUPPORTED_OUT_PRUNING_MODULES), \
                f"Cannot prune outgoing activations on this module. Only the following are supported " \
                f"{SUPPORTED_OUT_PRUNING_MODULES}"
        else:
            assert any(isinstance(module, t) for t in SUPPORTED_IN_PRUNING_MODULES), \
                f"Cannot prune incoming activations on this module. Only the following are supported " \
                f"{SUPPORTED_IN_PRUNING_MODULES}"
        if isinstance(module, _ConvNd) and module.groups != 1:
            raise NotImplementedError("structured pruning of grouped convolutions is not supported")
        indices = _as_index_array(indices)
        logger.info("Pruning %d units from %s (%s)", len(indices), module, direction)
        transposed = isinstance(module, _ConvTransposeNd)
        if direction == "out":
            self.prune_parameter(module, "weight", indices, axis=1 if transposed else 0)
            self.prune_parameter(module, "bias", indices, axis=0)
            _set_width(module, "out", module.weight.shape[1 if transposed else 0])
        else:
            if isinstance(module, (nn.Linear, _ConvNd)):
                self.prune_parameter(module, "weight", indices, axis=0 if transposed else 1)
                _set_width(module, "in", module.weight.shape[0 if transposed else 1])
            elif isinstance(module, _BatchNorm):
                self.prune_parameters(module, ["weight", "bias", "running_mean", "running_var"], indices, axis=0)
                module.num_features = module.running_mean.shape[0] if module.running_mean is not None \
                    else module.weight.shape[0]
            elif isinstance(module, _DropoutNd):
                self._adjust_dropout(module, indices, original_len)

    def prune_parameter(self, module, parameter_name, indices, axis=0):
        """Slice one parameter/buffer in place (Parameter identity preserved), with its grad
        and optimizer state."""
        self.prune_parameters(module, [parameter_name], indices, axis)

    def prune_parameters(self, module, names, indices, axis=0):
        """Slice several same-length tensors of ``module`` along ``axis`` in ONE gather launch."""
        with self._entry():
            indices = self._sync(_as_index_array(indices))
            return self._prune_parameters(module, names, indices, axis)

    def _prune_parameters(self, module, names, indices, axis=0):
        tensors, axes, sinks = [], [], []
        keep = None
        for name in names:
            param = getattr(module, name, None)
            if param is None:
                continue
            n = param.data.shape[axis]
            if keep is None:
                mask = np.ones(n, dtype=bool)
                if indices.size and (indices.max() >= n or indices.min() < -n):
                    # the reference raises here too (numpy fancy assignment, pruner.py:106-107):
                    # a bad score->index mapping must not silently mis-prune
                    raise IndexError(f"pruning index out of range for {name} with {n} entries along axis {axis}: "
                                     f"{indices[(indices >= n) | (indices < -n)].tolist()[:8]}")
                mask[indices] = False
                keep = torch.from_numpy(np.arange(n)[mask]).to(param.device)
            tensors.append(param.data)
            axes.append(axis)
            sinks.append(("data", param))
            if isinstance(param, torch.Tensor) and param.grad is not None:
                tensors.append(param.grad.data)
                axes.append(axis)
                sinks.append(("grad", param))
            if self.optimizer is not None and isinstance(param, nn.Parameter):
                for key, t in OptimizerPruner.state_tensors(self.optimizer, param):
                    tensors.append(t)
                    axes.append(axis)
                    sinks.append(("opt", (param, key)))
        if not tensors:
            return
        outs = ops.gather_multi(tensors, axes, keep)
        for (kind, target), new in zip(sinks, outs):
            if kind == "data":
                target.data = new
            elif kind == "grad":
                target.grad.data = new
            else:
                p, key = target
                self.optimizer.state[p][key] = new

    # ------------------------------------------------------------------ internals
    @contextlib.contextmanager
    def _entry(self):
        self._depth += 1
        try:
            yield
        finally:
            self._depth -= 1

    def _sync(self, indices: np.ndarray) -> np.ndarray:
        """R5: at the outermost public call of a data-parallel job every rank takes rank 0's
        indices (broadcast), and a rank whose own indices differed says so — every replica must
        prune identically, whichever API level the caller uses (prune_model / prune_module /
        prune_parameter(s)). Nested calls reuse the agreed indices (no extra collective)."""
        if self._depth > 1 or not self.sync_indices or pdist.get_world_size(self.group) <= 1:
            return indices
        agreed = np.asarray(pdist.broadcast_object(indices, 0, self.group), dtype=np.int64).reshape(-1)
        if not np.array_equal(agreed, indices):
            logger.warning("rank %d: pruning indices differ from rank 0's (%d vs %d units); using rank 0's",
                           pdist.get_rank(self.group), len(indices), len(agreed))
        return agreed

    def _adjust_dropout(self, module, indices, original_len):
        """Keep the expected number of active units: p *= 1 - pruned/original (pruner.py:117-127)."""
        if original_len is None:
            raise RuntimeError("Cannot adjust Dropout rate with 'original_len=None'")
        module.p *= (1.0 - len(indices) / original_len)

    def _nanify_hook(self, indices):
        """Forward hook writing NaN into output channels ``indices`` (simulated pruning)."""
        idx = _as_index_array(indices)

        def _hook(_, __, output):
            t = torch.as_tensor(idx, dtype=torch.long, device=output.device)
            if output.is_contiguous() and output.dtype == torch.float32:
                return ops.channel_fill_(output, t, float("nan"))
            return output.index_fill_(1, t, float("nan"))

        return _hook

    @staticmethod
    def _detect_nan_hook(probe=None):
        """Forward hook recording which input channels of a module carry NaNs: into ``probe``
        (a :class:`_ProbeRun`, what prune_model uses), or — called without one, as the
        reference's own tests do (test_pruner.py:77-120) — as ``_nan_indices`` /
        ``_activation_len`` attributes of the module."""

        def _hook(module, input, __):
            x = input[0]
            if probe is not None:
                probe.activation_len[module] = float(x.shape[1])
            else:
                setattr(module, "_activation_len", float(x.shape[1]))
            if x.dim() >= 2 and x.is_contiguous() and x.dtype == torch.float32:
                flags = ops.nan_channels(x)
            else:
                v = x
                while v.dim() > 2:
                    v = v.sum(-1)
                flags = torch.isnan(v.sum(0).flatten(0))
            indices = flags.nonzero().flatten(0).cpu().numpy()
            if len(indices) > 0:
                if probe is not None:
                    probe.nan_indices[module] = indices
                else:
                    setattr(module, "_nan_indices", indices)

        return _hook

    def _run_forward(self, x=None):
        d, b = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
        # see _AttributionMetric.set_deterministic for the ROCm/MIOpen exception
        if torch.version.hip is None or os.environ.get("TORCHPRUNER_DETERMINISTIC", "0") == "1":
            torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
        was_training = self.model.training
        self.model.eval()
        try:
            if x is None:
                x = torch.tensor(np.random.random((2,) + tuple(self.input_size))).float().to(self.device)
            with torch.no_grad():
                return self.model(x)
        finally:
            self.model.train(was_training)
            torch.backends.cudnn.deterministic = d
            torch.backends.cudnn.benchmark = b


class _ProbeRun:
    """What one NaN probe found, per cascading module (keyed by module object): the NaN input
    channels and the input width (for the Dropout rescale)."""

    def __init__(self):
        self.nan_indices = {}
        self.activation_len = {}


def _set_width(module, direction, n):
    if isinstance(module, nn.Linear):
        if direction == "out":
            module.out_features = n
        else:
            module.in_features = n
    elif isinstance(module, _ConvNd):
        if direction == "out":
            module.out_channels = n
        else:
            module.in_channels = n
