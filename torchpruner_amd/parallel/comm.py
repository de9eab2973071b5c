"""Pluggable collective backend.

Every ``group=`` argument of the package (metrics, ``parallel.dist`` helpers, ``PrunableDDP``
checks) accepts either a ``torch.distributed`` process group — the production path: RCCL over
xGMI on GPUs, gloo on CPUs — or a :class:`Communicator`. The in-process
:class:`LoopbackCommunicator` runs N ranks as N threads of one process; the data-parallel
attribution logic (batch sharding, the once-per-run score all-reduce, Shapley prefix sharding
and permutation broadcast) can then be unit-tested without spawning processes or opening
sockets. The reference has no distributed code at all.

Reductions are summed in rank order on the host, so a loopback run is bit-reproducible.
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

    def __init__(self, world_size: int, timeout: float = 120.0):
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

    def _exchange(self, value):
        self.hub.slots[self.rank] = value
        self.hub.barrier.wait()
        out = list(self.hub.slots)
        self.hub.barrier.wait()  # nobody overwrites a slot before everyone has read it
        return out

    def all_reduce_(self, t, op="sum"):
        vals = self._exchange(t.detach().to("cpu", copy=True))
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
        vals = self._exchange(t.detach().to("cpu", copy=True) if self.rank == src else None)
        t.copy_(vals[src].to(t.device))
        return t

    def all_gather(self, t):
        return [v.to(t.device) for v in self._exchange(t.detach().to("cpu", copy=True))]

    def all_gather_object(self, obj):
        return [copy.deepcopy(v) for v in self._exchange(obj)]

    def broadcast_object(self, obj, src=0):
        return copy.deepcopy(self._exchange(obj if self.rank == src else None)[src])

    def barrier(self):
        self._exchange(None)


def run_loopback(world_size: int, fn: Callable[..., Any], *args, timeout: float = 120.0) -> list:
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
