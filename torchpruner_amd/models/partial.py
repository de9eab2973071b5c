"""The ``forward_partial`` protocol (reference: experiments/models/cifar10.py:26-59).

``forward_partial(x, to_module=None, from_module=None)``: start right *after* ``from_module``
(exclusive) and return right *after* ``to_module`` (inclusive). Used by Shapley's fast path
and by the ablation studies to run only the layers downstream of a masked activation.
"""
from __future__ import annotations

from typing import Callable, Sequence, Union

import torch.nn as nn

Stage = Union[nn.Module, Callable]


def run_stages(stages: Sequence[Stage], x, to_module=None, from_module=None):
    """Run an ordered list of stages with the forward_partial semantics."""
    processing = from_module is None
    for stage in stages:
        if processing:
            x = stage(x)
            if to_module is not None and stage is to_module:
                return x
        elif stage is from_module:
            processing = True
    return x


class PartialForwardMixin:
    """Mixin for chain models: subclasses implement ``_stages()`` in execution order."""

    def _stages(self) -> Sequence[Stage]:  # pragma: no cover - abstract
        raise NotImplementedError

    def forward_partial(self, x, to_module=None, from_module=None):
        return run_stages(self._stages(), x, to_module=to_module, from_module=from_module)


class SequentialPartial(nn.Sequential, PartialForwardMixin):
    """``nn.Sequential`` that also speaks ``forward_partial`` (enables Shapley's fast path)."""

    def _stages(self):
        return list(self.children())


def with_forward_partial(seq: nn.Sequential) -> SequentialPartial:
    """Wrap an existing ``nn.Sequential`` (sharing its modules) into a SequentialPartial."""
    out = SequentialPartial()
    for name, m in seq.named_children():
        out.add_module(name, m)
    return out
