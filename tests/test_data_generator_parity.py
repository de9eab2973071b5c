"""The data generator is iterated exactly once per attribution pass (reference:
attributions.py:48,64), also when the engine selection needs the first batch's shape: a shuffling
DataLoader draws its sampler seed from the global torch RNG once, and a one-shot iterable loses
no batch."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, TensorDataset

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, ShapleyAttributionMetric,
                             TaylorAttributionMetric)


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(6, 8), nn.ReLU(), nn.Linear(8, 3))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(20, 6, generator=g), torch.randint(0, 3, (20,), generator=g)


def test_shuffling_loader_drawn_once_per_pass():
    model = _model()
    x, y = _data()
    for cls in (TaylorAttributionMetric, SensitivityAttributionMetric, APoZAttributionMetric):
        torch.manual_seed(5)
        dl = DataLoader(TensorDataset(x, y), batch_size=4, shuffle=True)
        cls(model, dl, F.cross_entropy, "cpu").run(model[0])
        after = torch.get_rng_state()
        torch.manual_seed(5)
        for _ in DataLoader(TensorDataset(x, y), batch_size=4, shuffle=True):
            pass
        assert torch.equal(after, torch.get_rng_state()), cls.__name__


def test_one_shot_iterable_loses_no_batch():
    model = _model()
    x, y = _data()
    batches = [(x[i:i + 4], y[i:i + 4]) for i in range(0, 20, 4)]
    ref = TaylorAttributionMetric(model, batches, F.cross_entropy, "cpu", reduction="none").run(model[0])
    got = TaylorAttributionMetric(model, iter(batches), F.cross_entropy, "cpu", reduction="none").run(model[0])
    assert got.shape == (20, 8)
    np.testing.assert_array_equal(got, ref)
    np.random.seed(3)
    ref = ShapleyAttributionMetric(model, batches, F.cross_entropy, "cpu", sv_samples=2, reduction="none").run(model[0])
    np.random.seed(3)
    got = ShapleyAttributionMetric(model, iter(batches), F.cross_entropy, "cpu", sv_samples=2,
                                   reduction="none").run(model[0])
    np.testing.assert_array_equal(got, ref)
