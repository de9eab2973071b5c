"""Synthetic, device-resident datasets (no torchvision / no network in this environment).

The reference trains and scores on CIFAR-10 / MNIST / FashionMNIST through torchvision
DataLoaders with ``num_workers=1`` (experiments/models/cifar10.py:80-161). Here data of the
same shapes is generated directly on the GPU, so attribution throughput is bound by the
engine and not by a host loader:

* :class:`DeviceLoader` — a fixed (x, y) tensor pair already on device, batched without
  copies; has ``.dataset`` (``len``) for Shapley and ``shard(rank, world)`` for
  data-parallel runs (round-robin whole batches, no foreign batch is ever touched).
* :class:`StreamLoader` — ImageNet-scale streams: batch ``i`` is regenerated on device from
  ``seed + i`` each time (nothing stored), so any rank can produce exactly its batches.
* ``teacher`` labels: ``y = argmax model(x)`` of a reference model, which gives a
  meaningful "top-1 retained after pruning" on random-init weights (top-1 = 100% before).
"""
from __future__ import annotations

import math
from typing import Callable, Optional

import torch

SHAPES = {
    "cifar10": ((3, 32, 32), 10),
    "mnist": ((1, 28, 28), 10),
    "fmnist": ((1, 28, 28), 10),
    "imagenet": ((3, 224, 224), 1000),
}


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


class DeviceLoader:
    """Iterate fixed on-device tensors in batches (like a non-shuffling DataLoader)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, drop_last: bool = False):
        assert x.shape[0] == y.shape[0]
        self.x, self.y = x, y
        self.batch_size = batch_size
        self.drop_last = drop_last
        self.dataset = _Len(x.shape[0])

    def __len__(self):
        n = self.x.shape[0]
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _batch(self, i):
        s = i * self.batch_size
        return self.x[s:s + self.batch_size], self.y[s:s + self.batch_size]

    def __iter__(self):
        for i in range(len(self)):
            yield self._batch(i)

    def shard(self, rank: int, world: int):
        for i in range(rank, len(self), world):
            x, y = self._batch(i)
            yield i, x, y


class ShardLoader:
    """One data-parallel rank's batches of a global batched data set, materialised on device:
    ``batches`` maps global batch index -> (x, y) for the indices this rank owns (round-robin,
    ``i % world == rank``). ``shard(rank, world)`` yields exactly those (each rank holds 1/world
    of the data instead of all of it); iterating it plainly is only valid when it owns all
    batches (world 1)."""

    def __init__(self, batches: dict, num_batches: int, batch_size: int, world: int = 1):
        self.batches = batches
        self.num_batches = num_batches
        self.batch_size = batch_size
        self.world = world
        self.dataset = _Len(num_batches * batch_size)

    @classmethod
    def build(cls, make_batch: Callable, num_batches: int, batch_size: int, rank: int = 0, world: int = 1):
        """``make_batch(i)`` -> (x, y) of global batch ``i`` (e.g. seeded from i); only this rank's
        batches are built."""
        return cls({i: make_batch(i) for i in range(rank, num_batches, world)}, num_batches, batch_size, world)

    def __len__(self):
        return self.num_batches

    @property
    def local_only(self) -> bool:
        """True when this loader was built for one rank of a multi-rank job (it holds only that
        rank's batches; every rank answers the same, so they agree on how to split work)."""
        return self.world > 1 or len(self.batches) != self.num_batches

    def __iter__(self):
        if len(self.batches) != self.num_batches:
            raise RuntimeError("ShardLoader holds one rank's batches; iterate it through shard(rank, world)")
        for i in range(self.num_batches):
            yield self.batches[i]

    def shard(self, rank: int, world: int):
        for i in range(rank, self.num_batches, world):
            if i not in self.batches:
                raise RuntimeError(f"batch {i} belongs to rank {rank} of {world} but was not built here")
            x, y = self.batches[i]
            yield i, x, y


class StreamLoader:
    """Deterministic on-device stream of ``num_batches`` random batches (nothing stored)."""

    def __init__(self, num_batches: int, batch_size: int, shape, num_classes: int, device, seed: int = 0,
                 labeler: Optional[Callable] = None, channels_last: bool = False):
        self.num_batches = num_batches
        self.batch_size = batch_size
        self.shape = tuple(shape)
        self.num_classes = num_classes
        self.device = torch.device(device)
        self.seed = seed
        self.labeler = labeler
        self.channels_last = channels_last
        self.dataset = _Len(num_batches * batch_size)

    def __len__(self):
        return self.num_batches

    def _batch(self, i):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed * 1_000_003 + i)
        x = torch.randn((self.batch_size,) + self.shape, generator=g, device=self.device)
        if self.channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        if self.labeler is not None:
            y = self.labeler(x)
        else:
            y = torch.randint(0, self.num_classes, (self.batch_size,), generator=g, device=self.device)
        return x, y

    def __iter__(self):
        for i in range(self.num_batches):
            yield self._batch(i)

    def shard(self, rank: int, world: int):
        for i in range(rank, self.num_batches, world):
            x, y = self._batch(i)
            yield i, x, y


def synthetic_dataset(name: str, n: int, device="cpu", seed: int = 0, teacher: Optional[torch.nn.Module] = None,
                      batch_for_teacher: int = 1024):
    """Return ``(x, y)`` of ``n`` samples shaped like dataset ``name`` on ``device``.

    With ``teacher`` the labels are the teacher's eval-mode argmax predictions.
    """
    shape, nc = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn((n,) + shape, generator=g).to(device)
    if teacher is None:
        y = torch.randint(0, nc, (n,), generator=g).to(device)
    else:
        y = teacher_labels(teacher, x, batch_for_teacher)
    return x, y


@torch.no_grad()
def teacher_labels(model: torch.nn.Module, x: torch.Tensor, batch: int = 1024) -> torch.Tensor:
    was = model.training
    model.eval()
    out = []
    for s in range(0, x.shape[0], batch):
        out.append(model(x[s:s + batch]).argmax(1))
    model.train(was)
    return torch.cat(out, 0)


class PrototypeTask:
    """A learnable synthetic classification task of a given image shape.

    Class ``c`` has a fixed smooth prototype image ``P_c`` (low-resolution Gaussian noise,
    bilinearly upsampled, unit variance); a sample is ``P_y + noise * N(0, 1)``. A CNN learns
    it in a few hundred steps, which makes "top-1 retained after pruning" meaningful without
    any dataset download (random-init networks predict one class for every input).
    """

    def __init__(self, shape=(3, 32, 32), num_classes=10, noise=1.0, seed=0, device="cpu", low_res=8,
                 modes_per_class=1, label_noise=0.0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        c, h, w = shape
        n_proto = num_classes * modes_per_class
        low = torch.randn(n_proto, c, low_res, low_res, generator=g)
        protos = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=False)
        protos = (protos - protos.mean((1, 2, 3), keepdim=True)) / protos.std((1, 2, 3), keepdim=True)
        self.protos = protos.to(device)
        self.noise = noise
        self.num_classes = num_classes
        self.modes_per_class = modes_per_class
        self.shape = tuple(shape)
        self.device = torch.device(device)
        self.label_noise = float(label_noise)

    def sample(self, n: int, seed: int):
        """``modes_per_class`` > 1 makes every class a mixture of several prototypes (a task that
        needs more of the network's capacity, so pruning a layer actually costs accuracy).
        ``label_noise`` = p replaces a fraction p of the labels (training and held-out alike) by a
        uniformly drawn class: irreducible error, so even a converged network tops out at
        (1 - p) + p / num_classes top-1 (p = 0.08, 10 classes: 0.928, the reference VGG16's CIFAR-10
        level, nbVGG:176) instead of saturating at 1.0."""
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        idx = torch.randint(0, self.num_classes * self.modes_per_class, (n,), generator=g, device=self.device)
        y = idx // self.modes_per_class
        x = self.protos[idx] + self.noise * torch.randn((n,) + self.shape, generator=g, device=self.device)
        if self.label_noise > 0:
            flip = torch.rand(n, generator=g, device=self.device) < self.label_noise
            y = torch.where(flip, torch.randint(0, self.num_classes, (n,), generator=g, device=self.device), y)
        return x, y

    def loader(self, n: int, batch_size: int, seed: int) -> "DeviceLoader":
        x, y = self.sample(n, seed)
        return DeviceLoader(x, y, batch_size)

    def stream(self, num_batches: int, batch_size: int, seed: int, channels_last: bool = False) -> "TaskStream":
        """Batches regenerated on device from ``(seed, i)`` (nothing stored; shardable)."""
        return TaskStream(self, num_batches, batch_size, seed, channels_last)


class TaskStream:
    """Deterministic on-device stream of :class:`PrototypeTask` batches; ``shard(rank, world)``
    yields only this rank's whole batches (data-parallel training / attribution)."""

    def __init__(self, task: PrototypeTask, num_batches: int, batch_size: int, seed: int, channels_last=False):
        self.task = task
        self.num_batches = num_batches
        self.batch_size = batch_size
        self.seed = seed
        self.channels_last = channels_last
        self.dataset = _Len(num_batches * batch_size)

    def __len__(self):
        return self.num_batches

    def _batch(self, i):
        x, y = self.task.sample(self.batch_size, self.seed * 1_000_003 + i)
        if self.channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        return x, y

    def __iter__(self):
        for i in range(self.num_batches):
            yield self._batch(i)

    def shard(self, rank: int, world: int):
        for i in range(rank, self.num_batches, world):
            x, y = self._batch(i)
            yield i, x, y


def loaders(name: str, n_train: int, n_val: int, batch_size: int, val_batch_size: int, device="cpu", seed: int = 0,
            teacher=None):
    """(train_loader, val_loader) of synthetic on-device data shaped like ``name``."""
    xt, yt = synthetic_dataset(name, n_train, device, seed, teacher)
    xv, yv = synthetic_dataset(name, n_val, device, seed + 1, teacher)
    return DeviceLoader(xt, yt, batch_size), DeviceLoader(xv, yv, val_batch_size)
