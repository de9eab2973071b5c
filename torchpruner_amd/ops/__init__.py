"""Device ops used by the attribution engine and the pruner.

Each function dispatches GPU tensors to the gfx950 HIP kernel registered under
``torch.ops.tpamd`` (csrc/) and CPU tensors to a plain-PyTorch reference of the same op.
The PyTorch bodies below are the numerics oracle the kernel tests compare against.
"""
from __future__ import annotations

from typing import Sequence

import torch

from ._native import available, backend, load, require, use_native

__all__ = [
    "available", "backend", "load", "require", "use_native",
    "REDUCE_MODES", "channel_reduce", "column_accumulate", "score_fold_", "channel_fill_", "nan_channels",
    "gather_multi", "prefix_mask", "shapley_scatter", "shapley_column", "cross_entropy",
]

REDUCE_MODES = {"taylor": 0, "taylor_signed": 1, "sensitivity": 2, "apoz": 3, "sum_grad": 4}


def _layout_ok(t: torch.Tensor) -> torch.Tensor:
    if t.is_contiguous():
        return t
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t
    return t.contiguous()


def _f32(t):
    if t is None:
        return None
    return _layout_ok(t if t.dtype == torch.float32 else t.float())


def channel_reduce(act: torch.Tensor | None, grad: torch.Tensor | None, mode: str) -> torch.Tensor:
    """Per-(sample, channel) score of a (B, C, ...) activation / gradient pair.

    taylor        |sum_s -(g*a)|      (taylor.py:40-46)
    taylor_signed  sum_s -(g*a)
    sensitivity    sum_s |g|          (sensitivity.py:27-29)
    apoz           sum_s [a > 0]      (apoz.py:31-33; a count for convs, not a fraction)
    sum_grad       sum_s g
    """
    m = REDUCE_MODES[mode]
    ref = act if act is not None else grad
    if use_native(ref):
        if act is not None and grad is not None:
            # both operands must share a memory layout for the kernel
            cl = ref.dim() == 4 and not ref.is_contiguous() and ref.is_contiguous(memory_format=torch.channels_last)
            fmt = torch.channels_last if cl else torch.contiguous_format
            act = act.float().contiguous(memory_format=fmt)
            grad = grad.float().contiguous(memory_format=fmt)
        return require().channel_reduce(_f32(act), _f32(grad), m)
    # PyTorch reference (reduced-precision operands are reduced in fp32)
    if act is not None and act.dtype in (torch.float16, torch.bfloat16):
        act = act.float()
    if grad is not None and grad.dtype in (torch.float16, torch.bfloat16):
        grad = grad.float()
    ref = act if act is not None else grad
    if mode in ("taylor", "taylor_signed"):
        v = -(grad * act)
    elif mode == "sensitivity":
        v = grad.abs()
    elif mode == "apoz":
        v = (act > 0).to(ref.dtype if ref.is_floating_point() else torch.float32)
    else:
        v = grad
    if v.dim() > 2:
        v = v.flatten(2).sum(-1)
    if mode == "taylor":
        v = v.abs()
    return v


def column_accumulate(v: torch.Tensor, acc_sum: torch.Tensor, acc_sq: torch.Tensor | None = None) -> None:
    """acc_sum += v.sum(0) (and acc_sq += (v*v).sum(0)) in float64, deterministic order."""
    if use_native(v):
        require().column_accumulate(v.float().contiguous(), acc_sum, acc_sq)
        return
    v64 = v.to(torch.float64)
    acc_sum += v64.sum(0)
    if acc_sq is not None:
        acc_sq += (v64 * v64).sum(0)


def score_fold_(Ts: Sequence[torch.Tensor], accs: Sequence[torch.Tensor | None], take_abs: bool, after: int) -> None:
    """For each (B, C) score slab T — or (R, B, C) partial slots, summed in slot order first —
    v = |T| (or T); acc += v.sum(0) in float64 (acc may be None); then ``after`` = 0 leaves T,
    1 writes v back into T (slot 0, other slots zeroed), 2 zeroes T. One launch for up to 16
    slabs (the fused engine folds every layer's scores at once)."""
    if len(Ts) == 0:
        return
    if use_native(*Ts):
        empty = torch.empty(0, dtype=torch.float64, device=Ts[0].device)
        require().score_fold_(list(Ts), [a if a is not None else empty for a in accs], bool(take_abs), int(after))
        return
    for T, a in zip(Ts, accs):
        tot = T.sum(0) if T.dim() == 3 else T
        v = tot.abs() if take_abs else tot
        if a is not None:
            a += v.double().sum(0)
        if after == 1:
            if T.dim() == 3:
                T[1:].zero_()
                T[0].copy_(v)
            else:
                T.copy_(v)
        elif after == 2:
            T.zero_()


def channel_fill_(x: torch.Tensor, idx, value: float) -> torch.Tensor:
    """In-place ``x.index_fill_(1, idx, value)`` for a contiguous (B, C, ...) tensor."""
    idx = torch.as_tensor(idx, dtype=torch.long, device=x.device).flatten()
    if use_native(x) and x.dtype == torch.float32 and x.is_contiguous():
        require().channel_fill_(x, idx, float(value))
        return x
    return x.index_fill_(1, idx, value)


def nan_channels(x: torch.Tensor) -> torch.Tensor:
    """Bool (C,) mask: channel c carries a NaN anywhere in the batch/trailing dims."""
    if use_native(x) and x.dtype == torch.float32:
        return require().nan_channels(x).bool()
    v = x
    while v.dim() > 2:
        v = v.sum(-1)
    return torch.isnan(v.sum(0).flatten(0))


def gather_multi(tensors: Sequence[torch.Tensor], axes: Sequence[int], keep: torch.Tensor) -> list[torch.Tensor]:
    """``[t.index_select(ax, keep) for t, ax]`` as ONE kernel launch per element size."""
    if len(tensors) == 0:
        return []
    if use_native(*tensors):
        return list(require().gather_multi(list(tensors), list(axes), keep.to(tensors[0].device, torch.long)))
    return [t.index_select(ax, keep.to(t.device, torch.long)) for t, ax in zip(tensors, axes)]


def prefix_mask(z: torch.Tensor, rank: torch.Tensor, p0: int, K: int) -> torch.Tensor:
    """Stack K prefix-masked copies of z: out[k] = z with channels of rank < p0+k zeroed."""
    if use_native(z) and z.dtype == torch.float32:
        return require().prefix_mask(_layout_ok(z), rank.to(z.device, torch.int32).contiguous(), int(p0), int(K))
    C = z.shape[1]
    ks = torch.arange(K, device=z.device).view(K, 1) + p0
    keep = (rank.to(z.device).view(1, C) >= ks).to(z.dtype)  # (K, C)
    shape = (K, 1, C) + (1,) * (z.dim() - 2)
    out = z.unsqueeze(0) * keep.view(shape)
    # multiplication would turn inf/NaN into NaN at masked positions; index_fill semantics are exact zeros
    out = torch.where(keep.view(shape) > 0, out, torch.zeros((), dtype=z.dtype, device=z.device))
    return out.reshape((K * z.shape[0],) + tuple(z.shape[1:]))


def shapley_scatter(L: torch.Tensor, perm: torch.Tensor, sv: torch.Tensor, row0: int, k0: int, scale: float) -> None:
    """sv[row0+b, perm[k0+k]] += (L[k+1,b] - L[k,b]) * scale for k < L.shape[0]-1."""
    if use_native(L):
        require().shapley_scatter(L.float().contiguous(), perm.to(L.device, torch.int32).contiguous(), sv,
                                  int(row0), int(k0), float(scale))
        return
    K = L.shape[0] - 1
    B = L.shape[1]
    d = (L[1:].double() - L[:-1].double()) * scale  # (K, B)
    cols = perm[k0:k0 + K].to(sv.device, torch.long)
    sv[row0:row0 + B, cols] += d.t()


def shapley_column(L: torch.Tensor, perm: torch.Tensor, sv_col: torch.Tensor, k0: int, scale: float) -> None:
    """sv_col[perm[k0+k]] += sum_b (L[k+1,b] - L[k,b]) * scale."""
    if use_native(L):
        require().shapley_column(L.float().contiguous(), perm.to(L.device, torch.int32).contiguous(), sv_col,
                                 int(k0), float(scale))
        return
    K = L.shape[0] - 1
    d = (L[1:].double() - L[:-1].double()).sum(1) * scale
    sv_col[perm[k0:k0 + K].to(sv_col.device, torch.long)] += d


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, gscale: float = 1.0, want_grad: bool = True):
    """Per-sample softmax cross-entropy and dL/dlogits * gscale (grad None if not wanted)."""
    if use_native(logits) and logits.dim() == 2:
        loss, grad = require().cross_entropy(logits.float(), target, float(gscale), bool(want_grad))
        return loss, (grad if want_grad else None)
    lf = logits.float()
    loss = torch.nn.functional.cross_entropy(lf, target.long(), reduction="none")
    grad = None
    if want_grad:
        p = torch.softmax(lf, 1)
        p[torch.arange(lf.shape[0]), target.long()] -= 1.0
        grad = p * gscale
    return loss, grad
