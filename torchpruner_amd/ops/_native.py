"""Loader for the in-tree gfx950 extension ``torchpruner_amd/_C.so``.

Policy (no silent fallbacks on a GPU box):
* GPU tensors always run the HIP kernels. If the extension cannot be loaded while a
  GPU is visible, :func:`require` raises with the load error.
* CPU tensors run the plain-PyTorch reference of each op (the numerics oracle used by
  the tests, and the path the CPU-only CI exercises).
* ``TORCHPRUNER_BACKEND=torch`` forces the PyTorch path everywhere; it exists only so the
  benchmark can measure the reference-semantics eager baseline on the same GPU.
* ``TORCHPRUNER_DEBUG_SYNC=1`` (debug mode, the analogue of ``AMD_SERIALIZE_KERNEL``): every
  native op is followed by a device synchronisation, so an asynchronous kernel fault is
  reported by the op that launched it (name and argument shapes) instead of a later one.
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
        _check_stamp()
        torch.ops.load_library(str(_LIB))
        _loaded = True
    except Exception as e:  # pragma: no cover - exercised on boxes without the build
        _error = e
    return _loaded


def _check_stamp():
    """Refuse a ``_C.so`` built from other sources than the tree it is loaded from (the build
    stamps the hash of every source and header into it, _build.source_hash). Build flags are
    stamped separately (_build.flag_hash): they depend on the build shell's environment
    (PYTORCH_ROCM_ARCH, TORCHPRUNER_HIPFLAGS), so a mismatch there only warns — a correct binary
    must not be refused because the loading shell's env differs."""
    from .. import _build
    if not (_build.CSRC / "kernels").is_dir():  # installed without sources: nothing to compare
        return
    want, got = _build.source_hash(), _build.stamped_hash(_LIB)
    if got != want:
        raise RuntimeError(f"stale native extension {_LIB}: built from sources {got}, this tree is {want}; "
                           "rebuild with `python -m torchpruner_amd._build` (or __graft_entry__.build())")
    fwant, fgot = _build.flag_hash(), _build.stamped_hash(_LIB, flags=True)
    if fgot != fwant:
        import warnings
        warnings.warn(f"native extension {_LIB} was built with other flags ({fgot}) than this environment "
                      f"implies ({fwant}: PYTORCH_ROCM_ARCH / TORCHPRUNER_HIPFLAGS / torch version); loading it",
                      RuntimeWarning, stacklevel=3)


def load_error():
    """Why the extension failed to load (None when loaded or not tried)."""
    return _error


def available() -> bool:
    return load()


class _SyncOps:
    """``torch.ops.tpamd`` proxy for TORCHPRUNER_DEBUG_SYNC=1: synchronise after every op."""

    def __init__(self, ns):
        self._ns = ns

    def __getattr__(self, name):
        op = getattr(self._ns, name)

        def call(*args, **kwargs):
            out = op(*args, **kwargs)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                shapes = [tuple(a.shape) if isinstance(a, torch.Tensor) else a for a in args]
                raise RuntimeError(f"tpamd.{name}{shapes} faulted: {e}") from e
            return out

        return call


def require():
    """Return ``torch.ops.tpamd`` or raise loudly (used on every GPU code path)."""
    if not load():
        raise RuntimeError(f"torchpruner_amd native extension unavailable: {_error!r}")
    if os.environ.get("TORCHPRUNER_DEBUG_SYNC", "0") == "1":
        return _SyncOps(torch.ops.tpamd)
    return torch.ops.tpamd


def use_native(*tensors) -> bool:
    """True when the op should run the HIP kernel for these tensors."""
    if backend() == "torch":
        return False
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)
