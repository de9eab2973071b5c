"""Pruning-graph utilities.

* :func:`find_best_module_for_attributions` — parity with the reference
  (torchpruner/utils/graph.py:9-34): walk ``model.modules()`` after ``module`` and move the
  evaluation point past any directly following BatchNorm / activation modules.
* :func:`get_vgg_pruning_graph` — parity with graph.py:37-61 for chain CNNs.
* :func:`get_resnet_pruning_graph` — new: residual-aware graph for bottleneck/basic-block
  ResNets (prune the block-internal convs, leave residual-tied convs alone).
* :func:`discover_cascade` — new: NaN-probe based consumer discovery for arbitrary graphs
  (SURVEY.md §7.3 hard part 6).
"""
from __future__ import annotations

import logging

import torch
import torch.nn as nn
from torch.nn.modules.activation import LeakyReLU, ReLU, ReLU6, RReLU, Sigmoid, Softplus, Tanh
from torch.nn.modules.batchnorm import _BatchNorm
from torch.nn.modules.conv import _ConvNd
from torch.nn.modules.dropout import _DropoutNd

logger = logging.getLogger("torchpruner")

ACTIVATIONS = (ReLU, ReLU6, RReLU, LeakyReLU, Sigmoid, Softplus, Tanh)


def find_best_module_for_attributions(model: nn.Module, module: nn.Module) -> nn.Module:
    """Return the last BatchNorm/activation that directly follows ``module``.

    Relies on registration order == execution order, exactly like the reference.
    Quirk preserved: if the chain of BN/activations runs to the end of ``modules()`` the
    original ``module`` is returned (reference graph.py:34).
    """
    modules = list(model.modules())
    try:
        current_idx = next(i for i, m in enumerate(modules) if m is module)
    except StopIteration:
        logger.error("Provided module is not in model")
        return module
    eval_module = module
    for next_module in modules[current_idx + 1:]:
        if isinstance(next_module, _BatchNorm):
            logger.info("BatchNorm detected: shifting evaluation after %s", next_module)
            eval_module = next_module
        elif isinstance(next_module, ACTIVATIONS):
            logger.info("Activation detected: shifting evaluation after %s", next_module)
            eval_module = next_module
        else:
            return eval_module
    return module


def get_vgg_pruning_graph(vgg: nn.Module):
    """List of ``(prunable_module, [cascading modules])`` for a chain CNN, last layer first.

    The cascade of a layer is ``[next Linear/Conv2d, BatchNorm2d..., Dropout...]`` — the same
    order the reference builds with append + reverse (graph.py:47-58) — and the final
    classifier is dropped.
    """
    pruning = []
    current = None
    for module in vgg.modules():
        if isinstance(module, (nn.Linear, nn.Conv2d)):
            if current is not None:
                pruning[-1][1].append(module)
                pruning[-1][1].reverse()
            current = module
            pruning.append((module, []))
        elif isinstance(module, (nn.BatchNorm2d, nn.Dropout)) and current is not None:
            pruning[-1][1].append(module)
    return pruning[::-1][1:]


def get_resnet_pruning_graph(model: nn.Module):
    """Residual-aware pruning graph for torchvision-style ResNets.

    For every residual block, the output channels of each internal conv (``conv1`` and, in a
    bottleneck, ``conv2``) can be pruned freely: the cut cascades into the block's BN and the
    next conv's input. The last conv of a block (``conv2`` of a BasicBlock / ``conv3`` of a
    Bottleneck) and the ``downsample`` convs write into the residual stream and stay intact.
    Returned last-block-first, like :func:`get_vgg_pruning_graph`.
    """
    graph = []
    for block in model.modules():
        convs = [(n, m) for n, m in block.named_children() if isinstance(m, nn.Conv2d) and n.startswith("conv")]
        if len(convs) < 2 or not any(n.startswith("bn") for n, _ in block.named_children()):
            continue
        convs.sort(key=lambda nm: int(nm[0][4:]) if nm[0][4:].isdigit() else 0)
        for i in range(len(convs) - 1):
            name, conv = convs[i]
            bn = getattr(block, "bn" + name[4:], None)
            nxt = convs[i + 1][1]
            cascade = [nxt] + ([bn] if isinstance(bn, _BatchNorm) else [])
            cascade.reverse()  # BN first, then the consumer conv (matches get_vgg_pruning_graph)
            graph.append((conv, cascade))
    return graph[::-1]


def discover_cascade(model: nn.Module, module: nn.Module, input_size, device=None, candidates=None):
    """Find the modules whose *input* channels depend on ``module``'s output channels.

    NaN-probe: nanify channel 0 of ``module``'s output, run one eval-mode no-grad forward on a
    random (2, *input_size) batch and report every Linear/Conv/BatchNorm/Dropout whose input
    picked up NaNs (the same trick the pruner uses, pruner.py:21-57, generalised to discover
    the cascade rather than requiring the user to spell it out).
    """
    if device is None:
        device = next(model.parameters()).device
    if candidates is None:
        candidates = [m for m in model.modules() if m is not module and
                      isinstance(m, (nn.Linear, _ConvNd, _BatchNorm, _DropoutNd))]
    found = []
    handles = []

    def nanify(_m, _i, out):
        out = out.clone()
        out[:, 0] = float("nan")
        return out

    def detect(m):
        def _h(_m, inp, _o):
            x = inp[0]
            v = x
            while v.dim() > 2:
                v = v.sum(-1)
            nan = torch.isnan(v.sum(0))
            # a direct consumer sees NaN in *some* input channels; anything past a
            # channel-mixing op sees NaN everywhere and is not part of the cascade
            if nan.any() and not nan.all():
                found.append(m)
        return _h

    handles.append(module.register_forward_hook(nanify))
    for m in candidates:
        handles.append(m.register_forward_hook(detect(m)))
    was_training = model.training
    model.eval()
    try:
        with torch.no_grad():
            model(torch.rand((2,) + tuple(input_size), device=device))
    finally:
        for h in handles:
            h.remove()
        model.train(was_training)
    seen = []
    for m in found:
        if not any(m is s for s in seen):
            seen.append(m)
    return seen
