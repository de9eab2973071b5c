"""Fused native execution engines (HIP kernels, no autograd) used by the attribution metrics
when the model/criterion/device allow it; everything else runs the generic hook path."""
from __future__ import annotations

import torch

from .fused_chain import FusedChainEngine, Plan, build_plan, criterion_is_cross_entropy, maybe_engine
from .resnet_engine import ResNetEngine, build_resnet_plan, maybe_resnet_engine

__all__ = ["FusedChainEngine", "Plan", "build_plan", "criterion_is_cross_entropy", "maybe_engine", "ResNetEngine",
           "build_resnet_plan", "maybe_resnet_engine", "native_logits", "invalidate"]


def invalidate(model) -> bool:
    """Drop the native engines cached for ``model`` (packed weights, autotuned plans, captured HIP
    graphs). The engines re-pack when a parameter's storage or version counter changes, which
    covers optimizer steps, ``load_state_dict``, pruning and in-place edits under ``no_grad``;
    in-place edits through ``param.data`` bypass the version counter, so call this after them.
    Also marks every cached training-conv weight pack stale (:func:`.train.invalidate_packs`).
    Returns True when something was cached."""
    from . import fused_chain, resnet_engine, train
    hit = train.invalidate_packs() > 0
    for cache in (fused_chain._ENGINES, resnet_engine._ENGINES):
        if model in cache:
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                # replays of the engine's captured graphs may still run on pipeline streams, and
                # dropping a graph returns its private pool to the allocator (as _bound_graph_cache)
                torch.cuda.synchronize()
            del cache[model]
            hit = True
    return hit


@torch.no_grad()
def native_logits(model, x: torch.Tensor):
    """Eval-mode logits of ``model`` on the native engines (fused chain: VGG-style CNNs and
    MLPs; ResNet engine), or None when neither applies (training mode, CPU, other models)."""
    if not isinstance(x, torch.Tensor) or not x.is_cuda or model.training:
        return None
    r = maybe_engine(model, [], None, x.device, need_ce=False, input_shape=tuple(x.shape))
    if r is not None:
        return r[0].forward(x)[0]
    eng = maybe_resnet_engine(model, [], x.device)
    if eng is not None:
        return eng.forward(x)
    return None
