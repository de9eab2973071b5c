"""dtype policy: exact fp32 by default; ``compute_dtype=torch.bfloat16``
is opt-in: on the GPU the fused engines run bf16-operand MFMA kernels (fp32 accumulation), on the
generic path (CPU, or float16) it autocasts the model's forward passes. Scores are still reduced
and accumulated in fp32/fp64, so they track the fp32 scores closely."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, ShapleyAttributionMetric,
                             TaylorAttributionMetric)
from torchpruner_amd.data import DeviceLoader


def _net():
    torch.manual_seed(0)
    return nn.Sequential(
        nn.Conv2d(3, 16, 3, padding=1), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2),
        nn.Conv2d(16, 32, 3, padding=1), nn.ReLU(), nn.Flatten(), nn.Linear(32 * 8 * 8, 10)).eval()


def _data(device="cpu", n=64):
    g = torch.Generator().manual_seed(1)
    return torch.randn(n, 3, 16, 16, generator=g).to(device), torch.randint(0, 10, (n,), generator=g).to(device)


def _rel(a, b):
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


@pytest.mark.parametrize("metric", [TaylorAttributionMetric, SensitivityAttributionMetric])
def test_bf16_gradient_scores_track_fp32(metric):
    model = _net()
    x, y = _data()
    mods = [model[0], model[4]]
    ref = metric(model, DeviceLoader(x, y, 16), F.cross_entropy, "cpu").run_many(mods, True)
    got = metric(model, DeviceLoader(x, y, 16), F.cross_entropy, "cpu",
                 compute_dtype=torch.bfloat16).run_many(mods, True)
    for a, r in zip(got, ref):
        assert a.dtype == np.float32 and a.shape == r.shape
        assert _rel(a, r) < 0.1
        assert np.corrcoef(a, r)[0, 1] > 0.98


def test_bf16_apoz_and_shapley_run():
    model = _net()
    x, y = _data(n=32)
    ref = APoZAttributionMetric(model, DeviceLoader(x, y, 16), F.cross_entropy, "cpu").run(model[0], find_best_evaluation_module=True)
    got = APoZAttributionMetric(model, DeviceLoader(x, y, 16), F.cross_entropy, "cpu",
                                compute_dtype=torch.bfloat16).run(model[0], find_best_evaluation_module=True)
    assert np.abs(got - ref).max() <= 0.05 * ref.max() + 1
    sv = ShapleyAttributionMetric(model, DeviceLoader(x, y, 16), F.cross_entropy, "cpu", sv_samples=2,
                                  compute_dtype=torch.bfloat16).run(model[4], find_best_evaluation_module=True)
    assert sv.shape == (32,) and np.isfinite(sv).all()


def test_compute_dtype_validated():
    model = _net()
    x, y = _data(n=8)
    with pytest.raises(AssertionError):
        TaylorAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, "cpu", compute_dtype=torch.int8)


@pytest.mark.gpu
def test_bf16_routes_to_fused_engine_on_gpu(monkeypatch):
    """On the GPU a bf16 compute dtype stays on the fused engine (bf16-operand MFMA kernels, fp32
    accumulation) instead of falling back to autocast on the generic path; its scores stay close
    to the fp32 engine's."""
    from torchpruner_amd.engine import fused_chain
    from torchpruner_amd.models import prunable_vgg16
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    x, y = torch.randn(64, 3, 32, 32, device=dev), torch.randint(0, 10, (64,), device=dev)
    convs = [m for m in model.features if isinstance(m, nn.Conv2d)]
    ref = TaylorAttributionMetric(model, DeviceLoader(x, y, 32), F.cross_entropy, dev).run_many(convs, True)
    calls = []
    orig = fused_chain.FusedChainEngine.taylor
    monkeypatch.setattr(fused_chain.FusedChainEngine, "taylor", lambda *a, **k: calls.append(1) or orig(*a, **k))
    got = TaylorAttributionMetric(model, DeviceLoader(x, y, 32), F.cross_entropy, dev,
                                  compute_dtype=torch.bfloat16).run_many(convs, True)
    assert len(calls) == 2  # one engine pass per batch
    for a, r in zip(got, ref):
        assert np.corrcoef(a, r)[0, 1] > 0.95
