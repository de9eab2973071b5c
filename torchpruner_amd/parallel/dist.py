"""Process-group plumbing for data-parallel attribution and prune->finetune.

One process per GPU, ``torch.distributed`` on RCCL (the ``"nccl"`` backend name IS RCCL
on ROCm) over xGMI, or gloo for CPU runs/tests. The reference has no distributed code at
all; the collectives introduced here are:

R1  all_reduce(SUM) of per-unit score sums + sample count     (one call per ``run()``)
R2  ordered all_gather of per-sample score slabs              (reduction "none"/callable)
R3  broadcast of Shapley permutations
R4  all_reduce(SUM) of Shapley accumulators
R5  broadcast of pruning indices (all ranks prune identically)
R8  all_reduce of correct/total counts in distributed test()

Attribution traffic is KB-scale and latency bound, so every payload is packed into one
flat buffer and reduced once per ``run()`` — never per batch.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Iterable, Iterator

import numpy as np
import torch
import torch.distributed as dist

from .comm import Communicator


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def _comm(group):
    """The Communicator behind ``group`` (None for torch process groups / the default group)."""
    return group if isinstance(group, Communicator) else None


def get_rank(group=None) -> int:
    if _comm(group):
        return group.rank
    return dist.get_rank(group) if is_dist() else 0


def get_world_size(group=None) -> int:
    if _comm(group):
        return group.world_size
    return dist.get_world_size(group) if is_dist() else 1


def init_distributed(backend: str | None = None, device: str | None = None) -> DistContext:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    Falls back to a single-process context when WORLD_SIZE is unset/1. GPU runs use one
    process per GPU with RCCL; CPU runs use gloo.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = (device != "cpu") and torch.cuda.is_available()
    if use_cuda:
        # TORCHPRUNER_SHARE_GPU=1 maps ranks onto the visible devices round-robin: a rehearsal
        # mode for multi-rank runs on a 1-GPU box (pair it with TORCHPRUNER_DIST_BACKEND=gloo,
        # RCCL refuses two ranks on one device)
        dev_index = local_rank % torch.cuda.device_count() if os.environ.get("TORCHPRUNER_SHARE_GPU") == "1" \
            else local_rank
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
    if backend is None:
        backend = os.environ.get("TORCHPRUNER_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    if world > 1 and not is_dist():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return DistContext(rank, world, local_rank, dev, backend)


def _comm_device(t: torch.Tensor, group=None) -> torch.device:
    """Device a tensor must live on for the active backend."""
    if not is_dist():
        return t.device
    be = dist.get_backend(group)
    if be == "nccl":
        return torch.device("cuda", torch.cuda.current_device()) if not t.is_cuda else t.device
    return torch.device("cpu")


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce that works for either backend (moves if needed)."""
    if get_world_size(group) == 1:
        return t
    if _comm(group):
        return group.all_reduce_(t, "sum")
    dev = _comm_device(t, group)
    if dev == t.device:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t
    tmp = t.to(dev)
    dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group)
    t.copy_(tmp.to(t.device))
    return t


def broadcast_object(obj: Any, src: int = 0, group=None) -> Any:
    if get_world_size(group) == 1:
        return obj
    if _comm(group):
        return group.broadcast_object(obj, src)
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]


def broadcast_tensor_(t: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if get_world_size(group) == 1:
        return t
    if _comm(group):
        return group.broadcast_(t, src)
    dev = _comm_device(t, group)
    tmp = t if dev == t.device else t.to(dev)
    dist.broadcast(tmp, src=src, group=group)
    if tmp is not t:
        t.copy_(tmp.to(t.device))
    return t


def all_max_int(v: int, group=None) -> int:
    """Max of a Python int over ranks (used to agree on shapes when a rank saw no data)."""
    if get_world_size(group) == 1:
        return int(v)
    if _comm(group):
        return max(group.all_gather_object(int(v)))
    vals = [None] * get_world_size(group)
    dist.all_gather_object(vals, int(v), group=group)
    return max(vals)


def all_max_float(x: float, group=None) -> float:
    """MAX of a Python float over ranks (any backend)."""
    if get_world_size(group) == 1:
        return float(x)
    if _comm(group):
        return float(group.all_reduce_(torch.tensor([float(x)], dtype=torch.float64), "max").item())
    t = torch.tensor([float(x)], dtype=torch.float64)
    dev = _comm_device(t, group)
    t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def barrier(group=None):
    if get_world_size(group) > 1:
        group.barrier() if _comm(group) else dist.barrier(group=group)


def all_gather_object(obj: Any, group=None) -> list:
    if get_world_size(group) == 1:
        return [obj]
    if _comm(group):
        return group.all_gather_object(obj)
    out = [None] * get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def state_digest(model: torch.nn.Module) -> str:
    """sha256 (16 hex) over every parameter and buffer of ``model`` (bytes, in state_dict order)."""
    import hashlib
    h = hashlib.sha256()
    for k, t in model.state_dict().items():
        h.update(k.encode() + str(t.dtype).encode())
        # raw bytes, dtype-agnostic (NumPy has no bfloat16)
        h.update(t.detach().cpu().contiguous().reshape(-1).view(torch.uint8).numpy().tobytes())
    return h.hexdigest()[:16]


def sync_module(model: torch.nn.Module, src: int = 0, group=None) -> dict:
    """Make every rank hold rank ``src``'s parameters and buffers, and report whether they
    already agreed: the digests are all-gathered BEFORE the broadcast (a replicated
    "deterministic" initialisation that diverged shows up as ``agreed_before: False``) and
    again after it (asserted equal). Data-parallel scores are only meaningful when every rank
    scores the same model."""
    world = get_world_size(group)
    mine = state_digest(model)
    if world == 1:
        return {"agreed_before": True, "digest": mine, "ranks": 1}
    before = all_gather_object(mine, group)
    with torch.no_grad():
        for t in model.state_dict().values():
            broadcast_tensor_(t, src, group)
    after = all_gather_object(state_digest(model), group)
    assert len(set(after)) == 1, f"model digests differ after broadcast: {after}"
    return {"agreed_before": len(set(before)) == 1, "digest": after[0], "ranks": world,
            "digests_before": before if len(set(before)) > 1 else None}


def gather_ordered_rows(slabs: list[tuple[int, torch.Tensor]], group=None) -> torch.Tensor:
    """All-gather per-batch ``(global_batch_index, (B_i, C) tensor)`` slabs from every rank
    and return the ``(sum B_i, C)`` concatenation in global batch order (R2).

    Metadata goes through one object all-gather; payload through one padded tensor
    all-gather.
    """
    world = get_world_size(group)
    local = sorted(slabs, key=lambda s: s[0])
    if world == 1:
        return torch.cat([s[1] for s in local], 0) if local else torch.empty(0)
    meta = [(i, t.shape[0]) for i, t in local]
    ncols = local[0][1].shape[1] if local else 0
    if _comm(group):
        metas = group.all_gather_object((meta, ncols))
    else:
        metas = [None] * world
        dist.all_gather_object(metas, (meta, ncols), group=group)
    ncols = max(m[1] for m in metas)
    rows = [sum(n for _, n in m[0]) for m in metas]
    maxrows = max(rows) if rows else 0
    ref = local[0][1] if local else torch.empty(0, ncols, dtype=torch.float32)
    dev = ref.device if _comm(group) else _comm_device(ref, group)
    buf = torch.zeros(maxrows, ncols, dtype=ref.dtype, device=dev)
    if local:
        mine = torch.cat([t for _, t in local], 0).to(dev)
        buf[: mine.shape[0]] = mine
    if _comm(group):
        outs = group.all_gather(buf)
    else:
        outs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
    pieces = []
    for r in range(world):
        off = 0
        for i, n in metas[r][0]:
            pieces.append((i, outs[r][off:off + n]))
            off += n
    pieces.sort(key=lambda p: p[0])
    return torch.cat([p[1] for p in pieces], 0).to(ref.device)


class ShardedBatches:
    """Iterate ``(global_batch_index, x, y)`` over the batches owned by one rank.

    Whole batches are assigned round-robin (batch ``i`` -> rank ``i % world``) so every
    batch keeps its own mean-loss scaling (Sensitivity/Taylor gradients carry 1/B from the
    mean; attributions.py:66) — the distributed scores equal the single-process ones.

    Fast paths avoid loading batches that another rank owns:
    * objects with a ``shard(rank, world)`` method (our on-device synthetic loaders);
    * ``torch.utils.data.DataLoader`` with a non-shuffling sampler: a per-rank loader over
      this rank's slice of the batch sampler is built (same workers / collate / pinning).
    Anything else is iterated in full and foreign batches are skipped.
    """

    def __init__(self, data_gen: Iterable, rank: int = 0, world_size: int = 1):
        self.data_gen = data_gen
        self.rank = rank
        self.world = world_size

    def __iter__(self) -> Iterator[tuple[int, Any, Any]]:
        dg, r, w = self.data_gen, self.rank, self.world
        if w == 1:
            for i, (x, y) in enumerate(dg):
                yield i, x, y
            return
        if hasattr(dg, "shard"):
            yield from dg.shard(r, w)
            return
        dl = _per_rank_dataloader(dg, r, w)
        if dl is not None:
            idxs, loader = dl
            for i, (x, y) in zip(idxs, loader):
                yield i, x, y
            return
        for i, (x, y) in enumerate(dg):
            if i % w == r:
                yield i, x, y


def _per_rank_dataloader(dg, rank, world):
    from torch.utils.data import DataLoader, SequentialSampler
    if not isinstance(dg, DataLoader) or dg.batch_sampler is None:
        return None
    sampler = getattr(dg.batch_sampler, "sampler", None)
    if not isinstance(sampler, SequentialSampler):
        return None
    batches = list(dg.batch_sampler)
    mine = [(i, b) for i, b in enumerate(batches) if i % world == rank]
    loader = DataLoader(dg.dataset, batch_sampler=[b for _, b in mine], num_workers=dg.num_workers,
                        collate_fn=dg.collate_fn, pin_memory=dg.pin_memory)
    return [i for i, _ in mine], loader


def split_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced split of ``range(total)`` (Shapley prefix-work sharding)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def seed_everything(seed: int):
    np.random.seed(seed)
    torch.manual_seed(seed)
