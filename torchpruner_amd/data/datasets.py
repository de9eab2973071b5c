"""Real datasets without torchvision: CIFAR-10 / MNIST / Fashion-MNIST from their original binary
files, resident in HBM, batched and augmented on the GPU.

The reference builds torchvision datasets + DataLoaders (experiments/models/cifar10.py:102-161,
mnist.py:62-82): a ``random_split`` of the training set into train / validation (1000 images by
default, or validation from the test set), training augmentation RandomHorizontalFlip +
RandomCrop(32, padding=4) + Normalize(ImageNet mean/std) for CIFAR-10, ToTensor only for MNIST,
``num_workers=1`` host workers, batch sizes 50/100/250 (CIFAR) and 100/1000/500 (MNIST).

Here (no network, no torchvision in this environment) the files are read from a local ``root``:

* CIFAR-10 binary version: ``data_batch_{1..5}.bin`` / ``test_batch.bin`` (each record = 1 label
  byte + 3072 pixel bytes, CHW), in ``root`` or ``root/cifar-10-batches-bin``;
* MNIST / Fashion-MNIST IDX files ``{train,t10k}-{images-idx3,labels-idx1}-ubyte[.gz]``, in
  ``root`` or ``root/MNIST/raw`` / ``root/FashionMNIST/raw``.

The uint8 images are uploaded ONCE (CIFAR-10 train: 150 MB of the 288 GB HBM); every batch is one
``tpamd.augment_u8`` launch (gather + flip + crop + normalise; a torch fallback on CPU) driven by
per-epoch seeded permutations and augmentation draws, so every data-parallel rank can produce
exactly its own batches (``shard``) with no host worker processes.
"""
from __future__ import annotations

import gzip
import math
import os
from typing import Optional

import numpy as np
import torch

from .. import ops

CIFAR_MEAN, CIFAR_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)  # cifar10.py:103-105


def _find(root: str, names, subdirs=("",)):
    for sub in subdirs:
        for n in names:
            p = os.path.join(root, sub, n)
            if os.path.exists(p):
                return p
    return None


def read_cifar10(root: str, train: bool = True):
    """(uint8 (N, 3, 32, 32), int64 (N,)) from the CIFAR-10 binary version."""
    names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    imgs, labels = [], []
    for n in names:
        p = _find(root, [n], ("", "cifar-10-batches-bin"))
        if p is None:
            raise FileNotFoundError(f"{n} not found under {root} (CIFAR-10 binary version; no download offline)")
        raw = np.fromfile(p, dtype=np.uint8).reshape(-1, 3073)
        labels.append(raw[:, 0].astype(np.int64))
        imgs.append(raw[:, 1:].reshape(-1, 3, 32, 32))
    return torch.from_numpy(np.concatenate(imgs)), torch.from_numpy(np.concatenate(labels))


def _read_idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    if data[0] != 0 or data[1] != 0 or data[2] != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    nd = data[3]
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(nd)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


def read_mnist(root: str, train: bool = True, fashion: bool = False):
    """(uint8 (N, 1, 28, 28), int64 (N,)) from the MNIST / Fashion-MNIST IDX files."""
    pre = "train" if train else "t10k"
    sub = ("", "FashionMNIST/raw" if fashion else "MNIST/raw", "raw")
    out = []
    for kind in ("images-idx3", "labels-idx1"):
        base = f"{pre}-{kind}-ubyte"
        p = _find(root, [base, base + ".gz"], sub)
        if p is None:
            raise FileNotFoundError(f"{base}[.gz] not found under {root} (no download offline)")
        out.append(_read_idx(p))
    imgs, labels = out
    return torch.from_numpy(imgs.copy()).unsqueeze(1), torch.from_numpy(labels.astype(np.int64))


def augment_batch(src: torch.Tensor, idx: torch.Tensor, aug: Optional[torch.Tensor], pad: int, mean: torch.Tensor,
                  inv_std: torch.Tensor) -> torch.Tensor:
    """Gather rows ``idx`` of the uint8 (N, C, H, W) ``src``, apply (dy, dx, flip) per image
    (RandomHorizontalFlip -> RandomCrop(H, padding=pad), zero fill) and normalise to fp32."""
    if ops.use_native(src):
        return ops.require().augment_u8(src, idx.contiguous(), aug.int().contiguous() if aug is not None else None,
                                        int(pad), mean, inv_std)
    x = src[idx].float() / 255.0
    if aug is not None:
        B, C, H, W = x.shape
        xp = torch.nn.functional.pad(x, (pad, pad, pad, pad))
        out = torch.empty_like(x)
        for b in range(B):
            dy, dx, flip = (int(v) for v in aug[b])
            img = xp[b].flip(-1) if flip else xp[b]  # flipping the padded image == padding the flipped one
            out[b] = img[:, dy:dy + H, dx:dx + W]
        x = out
    return (x - mean.view(1, -1, 1, 1)) * inv_std.view(1, -1, 1, 1)


class DeviceImageDataset:
    """uint8 images + labels resident on ``device`` with per-channel normalisation."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, device, mean=None, std=None):
        assert images.dtype == torch.uint8 and images.dim() == 4
        self.images = images.to(device).contiguous()
        self.labels = labels.to(device)
        C = images.shape[1]
        mean = mean if mean is not None else (0.0,) * C
        std = std if std is not None else (1.0,) * C
        self.mean = torch.tensor(mean, dtype=torch.float32, device=device)
        self.inv_std = 1.0 / torch.tensor(std, dtype=torch.float32, device=device)

    def __len__(self):
        return self.images.shape[0]

    def subset(self, indices: torch.Tensor) -> "DeviceSubset":
        return DeviceSubset(self, indices.to(self.images.device))


class DeviceSubset:
    def __init__(self, base: DeviceImageDataset, indices: torch.Tensor):
        self.base, self.indices = base, indices

    def __len__(self):
        return self.indices.numel()


class DeviceDataLoader:
    """Batches of a (subset of a) :class:`DeviceImageDataset` on the GPU.

    ``shuffle``: a new seeded permutation each epoch (identical on every rank); ``augment``:
    per-image crop offsets / flips drawn from the same seeded generator. ``shard(rank, world)``
    yields ``(global_batch_index, x, y)`` for this rank's whole batches only."""

    def __init__(self, data, batch_size: int, shuffle: bool = False, augment: bool = False, pad: int = 4,
                 seed: int = 0, drop_last: bool = False):
        self.base = data.base if isinstance(data, DeviceSubset) else data
        self.indices = data.indices if isinstance(data, DeviceSubset) else \
            torch.arange(len(data), device=self.base.images.device)
        self.batch_size, self.shuffle, self.augment, self.pad = batch_size, shuffle, augment, pad
        self.seed, self.drop_last, self.epoch = seed, drop_last, 0
        self.dataset = data

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __len__(self):
        n = self.indices.numel()
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _order(self):
        g = torch.Generator(device="cpu").manual_seed(self.seed * 1_000_003 + self.epoch)
        order = torch.randperm(self.indices.numel(), generator=g) if self.shuffle else \
            torch.arange(self.indices.numel())
        aug = None
        if self.augment:
            H, W = self.base.images.shape[2:]
            dy = torch.randint(0, 2 * self.pad + 1, (order.numel(),), generator=g)
            dx = torch.randint(0, 2 * self.pad + 1, (order.numel(),), generator=g)
            fl = torch.randint(0, 2, (order.numel(),), generator=g)
            aug = torch.stack([dy, dx, fl], 1).int().to(self.base.images.device)
        return self.indices[order.to(self.indices.device)], aug

    def _batch(self, order, aug, i):
        s = slice(i * self.batch_size, (i + 1) * self.batch_size)
        idx = order[s]
        x = augment_batch(self.base.images, idx, aug[s] if aug is not None else None, self.pad, self.base.mean,
                          self.base.inv_std)
        return x, self.base.labels[idx]

    def __iter__(self):
        order, aug = self._order()
        for i in range(len(self)):
            yield self._batch(order, aug, i)
        self.epoch += 1

    def shard(self, rank: int, world: int):
        order, aug = self._order()
        for i in range(rank, len(self), world):
            x, y = self._batch(order, aug, i)
            yield i, x, y
        self.epoch += 1


def _split(n: int, n_val: int, seed: int):
    g = torch.Generator(device="cpu").manual_seed(seed)
    perm = torch.randperm(n, generator=g)
    return perm[: n - n_val], perm[n - n_val:]


def get_dataset_and_loaders(name: str, root: str, device, val_split: int = 1000, val_from_test: bool = False,
                            batch_size: Optional[int] = None, val_batch_size: Optional[int] = None,
                            test_batch_size: Optional[int] = None, seed: int = 0):
    """(train_loader, validation_loader, test_loader) with the reference's split and batch sizes
    (cifar10.py:129-161 / mnist.py:62-82): ``name`` in {cifar10, mnist, fmnist}."""
    if name == "cifar10":
        xtr, ytr = read_cifar10(root, True)
        xte, yte = read_cifar10(root, False)
        mean, std, aug, bs = CIFAR_MEAN, CIFAR_STD, True, (50, 100, 250)
    elif name in ("mnist", "fmnist"):
        xtr, ytr = read_mnist(root, True, fashion=name == "fmnist")
        xte, yte = read_mnist(root, False, fashion=name == "fmnist")
        mean, std, aug, bs = None, None, False, (100, 1000, 500)
    else:
        raise ValueError(f"unknown dataset {name!r}")
    bs = (batch_size or bs[0], val_batch_size or bs[1], test_batch_size or bs[2])
    train = DeviceImageDataset(xtr, ytr, device, mean, std)
    # the validation split never sees training augmentation (as torchvision: val uses the train
    # transform in the reference only because random_split shares the dataset object; we keep
    # evaluation deterministic)
    test = DeviceImageDataset(xte, yte, device, mean, std)
    if val_from_test:
        te_idx, va_idx = _split(len(test), val_split, seed)
        val_set, test_set, train_set = test.subset(va_idx), test.subset(te_idx), train
    else:
        tr_idx, va_idx = _split(len(train), val_split, seed)
        train_set, val_set, test_set = train.subset(tr_idx), train.subset(va_idx), test
    return (DeviceDataLoader(train_set, bs[0], shuffle=True, augment=aug, seed=seed),
            DeviceDataLoader(val_set, bs[1], shuffle=False),
            DeviceDataLoader(test_set, bs[2], shuffle=name != "cifar10", seed=seed + 1))
