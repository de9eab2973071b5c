"""Real-dataset path (reference experiments/models/cifar10.py:102-161, mnist.py:62-82) on files
written here in the original binary formats (no dataset can be downloaded): readers, the
reference's train/val split and batch sizes, seeded shuffling / sharding, and the augmentation
(flip -> crop(padding) -> normalise) against an independent per-image torch formulation; the
HIP kernel (GPU) against the same oracle."""
import gzip
import os

import numpy as np
import pytest
import torch

from torchpruner_amd.data.datasets import (CIFAR_MEAN, CIFAR_STD, DeviceDataLoader, DeviceImageDataset, augment_batch,
                                           get_dataset_and_loaders, read_cifar10, read_mnist)


def _write_cifar(root, n_train_per_file=30, n_test=40, seed=0):
    rng = np.random.RandomState(seed)
    d = os.path.join(root, "cifar-10-batches-bin")
    os.makedirs(d)
    names = [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]
    for n in names:
        cnt = n_test if n.startswith("test") else n_train_per_file
        rec = np.zeros((cnt, 3073), np.uint8)
        rec[:, 0] = rng.randint(0, 10, cnt)
        rec[:, 1:] = rng.randint(0, 256, (cnt, 3072))
        rec.tofile(os.path.join(d, n))


def _write_idx(path, arr, gz):
    hdr = bytes([0, 0, 0x08, arr.ndim]) + b"".join(int(s).to_bytes(4, "big") for s in arr.shape)
    data = hdr + arr.astype(np.uint8).tobytes()
    if gz:
        with gzip.open(path + ".gz", "wb") as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def _write_mnist(root, n_train=1200, n_test=50, seed=0, gz=True):
    rng = np.random.RandomState(seed)
    d = os.path.join(root, "MNIST", "raw")
    os.makedirs(d)
    for pre, n in (("train", n_train), ("t10k", n_test)):
        _write_idx(os.path.join(d, f"{pre}-images-idx3-ubyte"), rng.randint(0, 256, (n, 28, 28)), gz)
        _write_idx(os.path.join(d, f"{pre}-labels-idx1-ubyte"), rng.randint(0, 10, n), gz)


def test_readers(tmp_path):
    _write_cifar(str(tmp_path / "c"))
    x, y = read_cifar10(str(tmp_path / "c"), True)
    assert x.shape == (150, 3, 32, 32) and x.dtype == torch.uint8 and y.shape == (150,) and int(y.max()) < 10
    raw = np.fromfile(str(tmp_path / "c" / "cifar-10-batches-bin" / "data_batch_2.bin"), np.uint8).reshape(-1, 3073)
    assert np.array_equal(x[30].numpy().reshape(-1), raw[0, 1:]) and int(y[30]) == raw[0, 0]
    xt, _ = read_cifar10(str(tmp_path / "c"), False)
    assert xt.shape == (40, 3, 32, 32)
    _write_mnist(str(tmp_path / "m"))
    xm, ym = read_mnist(str(tmp_path / "m"), True)
    assert xm.shape == (1200, 1, 28, 28) and ym.shape == (1200,)
    with pytest.raises(FileNotFoundError):
        read_mnist(str(tmp_path / "m"), True, fashion=True)


def _oracle(img_u8, dy, dx, flip, pad, mean, std):
    """torchvision order: flip the PIL image, pad with 0, crop at (dy, dx), ToTensor, Normalize."""
    x = img_u8.float() / 255.0
    if flip:
        x = x.flip(-1)
    C, H, W = x.shape
    p = torch.zeros(C, H + 2 * pad, W + 2 * pad)
    p[:, pad:pad + H, pad:pad + W] = x
    x = p[:, dy:dy + H, dx:dx + W]
    return (x - torch.tensor(mean).view(-1, 1, 1)) / torch.tensor(std).view(-1, 1, 1)


def _check_augment(dev):
    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, 256, (9, 3, 32, 32), generator=g, dtype=torch.uint8)
    ds = DeviceImageDataset(src, torch.zeros(9, dtype=torch.long), dev, CIFAR_MEAN, CIFAR_STD)
    idx = torch.tensor([4, 0, 8, 4, 2], device=dev)
    aug = torch.tensor([[0, 0, 0], [8, 8, 1], [4, 4, 1], [3, 7, 0], [8, 0, 1]], dtype=torch.int32, device=dev)
    out = augment_batch(ds.images, idx, aug, 4, ds.mean, ds.inv_std).cpu()
    for b in range(5):
        ref = _oracle(src[int(idx[b])], *(int(v) for v in aug[b]), 4, CIFAR_MEAN, CIFAR_STD)
        torch.testing.assert_close(out[b], ref, rtol=1e-5, atol=1e-5)
    plain = augment_batch(ds.images, idx, None, 4, ds.mean, ds.inv_std).cpu()
    torch.testing.assert_close(plain[1], _oracle(src[0], 4, 4, 0, 4, CIFAR_MEAN, CIFAR_STD))


def test_augment_cpu():
    _check_augment(torch.device("cpu"))


@pytest.mark.gpu
def test_augment_kernel(cuda):
    _check_augment(cuda)


def test_reference_split_and_loaders(tmp_path):
    _write_cifar(str(tmp_path / "c"), n_train_per_file=300, n_test=500)
    tr, va, te = get_dataset_and_loaders("cifar10", str(tmp_path / "c"), "cpu")
    assert (len(tr.dataset), len(va.dataset), len(te.dataset)) == (1500 - 1000, 1000, 500)
    assert (tr.batch_size, va.batch_size, te.batch_size) == (50, 100, 250)  # cifar10.py:147-158
    seen = torch.cat([y for _, y in va])
    assert seen.shape == (1000,)
    # train/val disjoint and together the whole training set
    all_idx = torch.cat([tr.indices, va.indices]).sort().values
    assert torch.equal(all_idx, torch.arange(1500))
    # seeded epochs: same order on every "rank", a new order next epoch
    e0 = [y for _, y in tr]
    tr.set_epoch(0)
    again = [y for _, y in tr]
    assert all(torch.equal(a, b) for a, b in zip(e0, again))
    tr.set_epoch(0)
    s0 = list(tr.shard(0, 2))
    tr.set_epoch(0)
    s1 = list(tr.shard(1, 2))
    got = {i: (x, y) for i, x, y in s0 + s1}
    assert sorted(got) == list(range(len(tr)))
    for i, y in enumerate(e0):  # the shards are exactly the single-process epoch
        assert torch.equal(got[i][1], y)
    _write_mnist(str(tmp_path / "m"))
    tr, va, te = get_dataset_and_loaders("mnist", str(tmp_path / "m"), "cpu")
    assert (len(tr.dataset), len(va.dataset), tr.batch_size, va.batch_size, te.batch_size) == (200, 1000, 100, 1000, 500)
    x, y = next(iter(tr))
    assert x.shape == (100, 1, 28, 28) and x.dtype == torch.float32 and float(x.max()) <= 1.0


def test_loader_drives_attribution(tmp_path):
    """A DeviceDataLoader is a drop-in data_generator for the metrics (incl. Shapley's len())."""
    import torch.nn as nn
    import torch.nn.functional as F
    from torchpruner_amd import APoZAttributionMetric
    _write_mnist(str(tmp_path / "m"), n_train=1100)
    _, va, _ = get_dataset_and_loaders("mnist", str(tmp_path / "m"), "cpu", val_batch_size=250)
    model = nn.Sequential(nn.Flatten(), nn.Linear(784, 16), nn.ReLU(), nn.Linear(16, 10)).eval()
    s = APoZAttributionMetric(model, va, F.cross_entropy, "cpu").run(model[1])
    assert s.shape == (16,) and np.isfinite(s).all()
    assert isinstance(va, DeviceDataLoader) and len(va.dataset) == 1000
