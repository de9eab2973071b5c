"""Pluggable collective backend.

The ``group=`` arguments of the attribution metrics, the ``Pruner`` index broadcast (R5) and
the ``parallel.dist`` helpers accept either a ``torch.distributed`` process group — the
production path: RCCL over xGMI on GPUs, gloo on CPUs — or a :class:`Communicator`.
``PrunableDDP`` and ``utils.train.test`` take torch process groups only (DDP itself needs one). The in-process
:class:`LoopbackCommunicator` runs N ranks as N threads of one process; the data-parallel
attribution logic (batch sharding, the once-per-run score all-reduce, Shapley prefix sharding
and permutation broadcast) can then be unit-tested without spawning processes or opening
sockets. The reference has no distributed code at all.

Reductions are summed in rank order on the host, so a loopback run is bit-reproducible.

Limitation: loopback ranks are threads of ONE process, so they share process-global state —
NumPy's global RNG (Shapley permutations are drawn on rank 0 only and broadcast, so this is
safe there), the ``torch.backends.cudnn`` flags the metrics save/restore, torch's RNG. Tests are
valid only while no rank's result depends on such state being private.
"""
from __future__ import annotations

import copy
import threading
from typing import Any, Callable

import torch


class Communicator:
    """Collective interface used when a ``group=`` argument is not a torch process group."""

    rank: int = 0
    world_size: int = 1

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> list[torch.Tensor]:
        raise NotImplementedError

    def all_gather_object(self, obj: Any) -> list:
        raise NotImplementedError

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError


class LoopbackHub:
    """Rendezvous shared by the ``world_size`` threads of one loopback job."""

    def __init__(self, world_size: int, timeout: float | None = None):
        """``timeout`` (seconds) bounds every wait of a collective; None (default) waits for as
        long as the slowest rank computes between two collectives."""
        self.world_size = world_size
        self.slots: list = [None] * world_size
        self.barrier = threading.Barrier(world_size, timeout=timeout)


class LoopbackCommunicator(Communicator):
    """One rank of an in-process job: every collective is a two-phase exchange through the
    hub's slots (publish, wait, read all, wait)."""

    def __init__(self, hub: LoopbackHub, rank: int):
        assert 0 <= rank < hub.world_size
        self.hub = hub
        self.rank = rank
        self.world_size = hub.world_size

    def _exchange(self, value, tag):
        """Publish ``value``; every rank must call the same collective (``tag``: op name and,
        for tensors, shape/dtype) — a mismatch raises on every rank instead of mixing payloads."""
        self.hub.slots[self.rank] = (tag, value)
        self.hub.barrier.wait()
        out = list(self.hub.slots)
        self.hub.barrier.wait()  # nobody overwrites a slot before everyone has read it
        tags = [o[0] for o in out]
        if any(t != tags[0] for t in tags):
            raise RuntimeError(f"mismatched collectives across loopback ranks: {tags}")
        return [o[1] for o in out]

    @staticmethod
    def _ttag(op, t):
        return (op, tuple(t.shape), t.dtype)

    def all_reduce_(self, t, op="sum"):
        vals = self._exchange(t.detach().to("cpu", copy=True), self._ttag("all_reduce_" + op, t))
        acc = vals[0].clone()
        for v in vals[1:]:  # fixed rank order: deterministic
            if op == "sum":
                acc += v
            elif op == "max":
                acc = torch.maximum(acc, v)
            else:
                raise ValueError(f"unsupported op {op!r}")
        t.copy_(acc.to(t.device))
        return t

    def broadcast_(self, t, src=0):
        vals = self._exchange(t.detach().to("cpu", copy=True) if self.rank == src else None,
                              self._ttag(f"broadcast_{src}", t))
        t.copy_(vals[src].to(t.device))
        return t

    def all_gather(self, t):
        # every rank owns its outputs: an in-place edit on one rank never reaches another
        return [v.to(t.device, copy=True) for v in self._exchange(t.detach().to("cpu", copy=True),
                                                                   self._ttag("all_gather", t))]

    def all_gather_object(self, obj):
        return [copy.deepcopy(v) for v in self._exchange(obj, ("all_gather_object",))]

    def broadcast_object(self, obj, src=0):
        return copy.deepcopy(self._exchange(obj if self.rank == src else None, ("broadcast_object", src))[src])

    def barrier(self):
        self._exchange(None, ("barrier",))


def run_loopback(world_size: int, fn: Callable[..., Any], *args, timeout: float | None = None) -> list:
    """Run ``fn(comm, *args)`` on ``world_size`` threads, one :class:`LoopbackCommunicator`
    each; returns the per-rank results. An exception on any rank aborts the rendezvous (the
    other ranks fail fast instead of waiting out the timeout) and is re-raised."""
    hub = LoopbackHub(world_size, timeout)
    results: list = [None] * world_size
    errors: list = [None] * world_size

    def body(r):
        try:
            results[r] = fn(LoopbackCommunicator(hub, r), *args)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e
            hub.barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world_size)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    first = next((e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
    if first is None:
        first = next((e for e in errors if e is not None), None)
    if first is not None:
        raise first
    return results
