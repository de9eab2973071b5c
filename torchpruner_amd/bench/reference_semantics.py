"""Reference-semantics eager baseline, measured on the same GPU as our engine.

The reference publishes no throughput numbers, so the comparison point for
"attribution images/sec" is the reference algorithm executed faithfully in eager PyTorch:

* one ``run()`` per module: scoring all prunable layers means one full data pass per layer
  (reference taylor.py:18-28 + attributions.py:58-68);
* a forward hook that stores a full ``clone()`` of the activation (taylor.py:31-36);
* the deprecated non-full ``register_backward_hook`` (taylor.py:21);
* a *full* backward (weight gradients included; ``param.grad`` accumulates);
* per-batch ``.detach().cpu().numpy()`` + ``np.concatenate`` on the host (taylor.py:46-48);
* ``np.mean`` over samples at the end (attributions.py:91-106).

This is a behavioural re-implementation written for benchmarking/parity tests, not the
reference's code. It is never used by the library itself.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch


def reference_taylor_scores(model, loader, criterion, device, eval_module, signed=False):
    """Taylor scores of one evaluation module with the reference's execution strategy."""
    store = {}

    def fwd(_m, _i, out):
        with torch.no_grad():
            store["act"] = out.detach().clone()

    def bwd(_m, _gi, go):
        t = -1.0 * (go[0] * store["act"])
        if t.dim() > 2:
            t = t.flatten(2).sum(-1)
        if not signed:
            t = t.abs()
        v = t.detach().cpu().numpy()
        store["acc"] = v if "acc" not in store else np.concatenate((store["acc"], v), 0)

    h1 = eval_module.register_forward_hook(fwd)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        h2 = eval_module.register_backward_hook(bwd)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for x, y in loader:
                x, y = x.to(device), y.to(device)
                loss = criterion(model(x), y)
                loss.backward()
    finally:
        h1.remove()
        h2.remove()
    return np.mean(store["acc"], 0)


def reference_taylor_all(model, loader, criterion, device, eval_modules, signed=False):
    """Score every module the reference way: one full data pass per module."""
    return [reference_taylor_scores(model, loader, criterion, device, m, signed) for m in eval_modules]
