"""Loader for the in-tree gfx950 extension ``torchpruner_amd/_C.so``.

Policy (no silent fallbacks on a GPU box):
* GPU tensors always run the HIP kernels. If the extension cannot be loaded while a
  GPU is visible, :func:`require` raises with the load error.
* CPU tensors run the plain-PyTorch reference of each op (the numerics oracle used by
  the tests, and the path the CPU-only CI exercises).
* ``TORCHPRUNER_BACKEND=torch`` forces the PyTorch path everywhere; it exists only so the
  benchmark can measure the reference-semantics eager baseline on the same GPU.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

_LIB = Path(__file__).resolve().parent.parent / "_C.so"
_loaded = False
_error: Exception | None = None


def backend() -> str:
    return os.environ.get("TORCHPRUNER_BACKEND", "hip").lower()


def load() -> bool:
    """Load ``_C.so`` once. Returns True when the ``torch.ops.tpamd`` namespace is live."""
    global _loaded, _error
    if _loaded:
        return True
    if _error is not None:
        return False
    try:
        if not _LIB.exists():
            raise FileNotFoundError(
                f"{_LIB} not built; run `python -m torchpruner_amd._build` (or __graft_entry__.build())")
        torch.ops.load_library(str(_LIB))
        _loaded = True
    except Exception as e:  # pragma: no cover - exercised on boxes without the build
        _error = e
    return _loaded


def available() -> bool:
    return load()


def require():
    """Return ``torch.ops.tpamd`` or raise loudly (used on every GPU code path)."""
    if not load():
        raise RuntimeError(f"torchpruner_amd native extension unavailable: {_error!r}")
    return torch.ops.tpamd


def use_native(*tensors) -> bool:
    """True when the op should run the HIP kernel for these tensors."""
    if backend() == "torch":
        return False
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)
