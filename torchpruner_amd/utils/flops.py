"""Parameter / FLOP counter (replaces the reference's ``thop.profile`` use in
experiments/utils/utils.py:30-36; thop is not available in this image).

MAC counting rules follow thop's: Conv = out_elems * (Cin/groups * kh*kw + bias),
Linear = out_elems * in_features, BatchNorm = 2 * elems (affine), everything else 0.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn.modules.batchnorm import _BatchNorm
from torch.nn.modules.conv import _ConvNd


def count_parameters(model: nn.Module, trainable_only: bool = False) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad or not trainable_only)


def count_flops(model: nn.Module, input_size, device=None, batch: int = 2) -> tuple[int, int]:
    """Return ``(flops_per_sample, params)`` with flops = 2 * MACs for one sample.

    Runs one eval-mode no-grad forward on a ``(batch, *input_size)`` random input (batch >= 2
    so BatchNorm in train mode would also work, as the reference notes).
    """
    if device is None:
        p = next(model.parameters(), None)
        device = p.device if p is not None else "cpu"
    macs = [0]

    def hook(m, inp, out):
        if isinstance(m, _ConvNd):
            k = m.weight[0].numel()  # Cin/groups * prod(kernel)
            macs[0] += out.numel() * (k + (1 if m.bias is not None else 0))
        elif isinstance(m, nn.Linear):
            macs[0] += out.numel() * m.in_features
        elif isinstance(m, _BatchNorm):
            macs[0] += 2 * inp[0].numel()

    handles = [m.register_forward_hook(hook) for m in model.modules()
               if isinstance(m, (_ConvNd, nn.Linear, _BatchNorm))]
    was_training = model.training
    model.eval()
    try:
        with torch.no_grad():
            model(torch.randn((batch,) + tuple(input_size), device=device))
    finally:
        for h in handles:
            h.remove()
        model.train(was_training)
    return int(2 * macs[0] // batch), count_parameters(model)
