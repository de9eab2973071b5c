"""Golden-value parity with the reference suite (torchpruner/tests/test_attributions.py).

The expectations (not the code) are ported: the 2-4-1 "max" ReLU network of
test_attributions.py:19-45 with hand-set weights, batch size 1, MSE loss. Every test runs on
CPU (PyTorch path) and, marked ``gpu``, on the MI355X (HIP kernels).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, TensorDataset

from torchpruner.attributions import (
    APoZAttributionMetric,
    RandomAttributionMetric,
    SensitivityAttributionMetric,
    ShapleyAttributionMetric,
    TaylorAttributionMetric,
    WeightNormAttributionMetric,
)

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        from torchpruner_amd import ops
        ops.require()
    return torch.device(name)


def max_model(device, version=1):
    x = np.array([[0, 1], [1, 0], [1, 2], [2, 1]])
    y = np.array([[np.max(xi)] for xi in x])
    x = torch.tensor(x).float().to(device)
    y = torch.tensor(y).float().to(device)
    w1 = torch.tensor([[-0.5, 1.0, 1.0, 1.0], [0.5, -1.0, 1.0, 1.0]]).float()
    if version == 1:
        w2 = torch.tensor([[1], [0.5], [0.5], [0.0]]).float()
    else:
        w2 = torch.tensor([[1], [0.5], [0.5], [-0.1]]).float()
    linear1 = nn.Linear(2, 4, bias=False)
    linear1.weight.data = torch.t(w1).to(device)
    linear2 = nn.Linear(4, 2, bias=False)
    linear2.weight.data = torch.t(w2).to(device)
    model = nn.Sequential(linear1, nn.ReLU(), linear2).to(device)
    return x, y, model


def loader(x, y):
    return DataLoader(TensorDataset(x, y), batch_size=1, shuffle=False)


@pytest.mark.parametrize("dev", DEVICES)
def test_max_model(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    np.testing.assert_array_almost_equal(y.cpu().numpy(), model(x).detach().cpu().numpy())


@pytest.mark.parametrize("dev", DEVICES)
def test_random(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    attr = RandomAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    assert list(attr.shape) == [4]


@pytest.mark.parametrize("dev", DEVICES)
def test_weight_norm(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    attr = WeightNormAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [1, 2, 2, 2])


@pytest.mark.parametrize("dev", DEVICES)
def test_apoz(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    attr = APoZAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    assert attr.dtype == np.float32
    np.testing.assert_array_almost_equal(attr, [0.5, 0.5, 1, 1])


@pytest.mark.parametrize("dev", DEVICES)
def test_sensitivity(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    attr = SensitivityAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [0.0, 0.0, 0.0, 0.0])


@pytest.mark.parametrize("dev", DEVICES)
def test_taylor(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    attr = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [0.0, 0.0, 0.0, 0.0])


@pytest.mark.parametrize("dev", DEVICES)
def test_sv(dev):
    d = _dev(dev)
    np.random.seed(0)
    x, y, model = max_model(d)
    a = ShapleyAttributionMetric(model, loader(x, y), F.mse_loss, d, sv_samples=1000)
    attr = a.run(list(model.children())[0])
    assert list(attr.shape) == [4]
    np.testing.assert_array_almost_equal(attr, [0.37, 0.37, 1.7, 0.0], decimal=1)


@pytest.mark.parametrize("dev", DEVICES)
def test_sensitivity_2(dev):
    d = _dev(dev)
    x, y, model = max_model(d, version=2)
    attr = SensitivityAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [0.2, 0.1, 0.2, 0.04])


@pytest.mark.parametrize("dev", DEVICES)
def test_taylor_2(dev):
    d = _dev(dev)
    x, y, model = max_model(d, version=2)
    attr = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, d).run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [0.1, 0.1, 0.5, 0.1])


@pytest.mark.parametrize("dev", DEVICES)
def test_taylor_2_signed(dev):
    d = _dev(dev)
    x, y, model = max_model(d, version=2)
    a = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, d, signed=True)
    attr = a.run(list(model.children())[0])
    np.testing.assert_array_almost_equal(attr, [0.1, 0.1, 0.5, -0.1])


@pytest.mark.parametrize("dev", DEVICES)
def test_find_best_evaluation_module(dev):
    d = _dev(dev)
    x, y, _ = max_model(d, version=2)
    model = nn.Sequential(nn.Linear(3, 2), nn.BatchNorm1d(2), nn.ReLU(), nn.Linear(2, 1)).to(d)
    for A in [TaylorAttributionMetric, SensitivityAttributionMetric, ShapleyAttributionMetric, APoZAttributionMetric]:
        a = A(model, loader(x, y), F.mse_loss, d)
        assert a.find_evaluation_module(list(model.children())[0], find_best_evaluation_module=True) \
            is list(model.children())[2]
    for A in [WeightNormAttributionMetric, RandomAttributionMetric]:
        a = A(model, loader(x, y), F.mse_loss, d)
        assert a.find_evaluation_module(list(model.children())[0], find_best_evaluation_module=True) \
            is list(model.children())[0]


@pytest.mark.parametrize("dev", DEVICES)
def test_run_all_with_find_best_evaluation_module(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    for A in [TaylorAttributionMetric, SensitivityAttributionMetric, APoZAttributionMetric,
              WeightNormAttributionMetric]:
        a = A(model, loader(x, y), F.mse_loss, d)
        attr = a.run(list(model.children())[0], find_best_evaluation_module=False)
        attr_best = a.run(list(model.children())[0], find_best_evaluation_module=True)
        np.testing.assert_array_almost_equal(attr, attr_best)


@pytest.mark.parametrize("dev", DEVICES)
def test_run_all_with_find_best_evaluation_module_2(dev):
    d = _dev(dev)
    x, y, model = max_model(d)
    for A in [TaylorAttributionMetric, SensitivityAttributionMetric, APoZAttributionMetric,
              WeightNormAttributionMetric, RandomAttributionMetric, ShapleyAttributionMetric]:
        a = A(model, loader(x, y), F.mse_loss, d)
        attr_best = a.run(list(model.children())[0], find_best_evaluation_module=True)
        assert list(attr_best.shape) == [4]


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("reduction", ["none", "sum", "callable"])
def test_reductions(dev, reduction):
    """Per-sample slabs come back in data order; sum/mean/callable agree with them."""
    d = _dev(dev)
    x, y, model = max_model(d, version=2)
    red = (lambda a: np.mean(a, 0) + 2 * np.std(a, 0)) if reduction == "callable" else reduction
    a = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, d, signed=True, reduction=red)
    attr = a.run(list(model.children())[0])
    per = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, d, signed=True, reduction="none") \
        .run(list(model.children())[0])
    assert per.shape == (4, 4)
    np.testing.assert_array_almost_equal(per.mean(0), [0.1, 0.1, 0.5, -0.1])
    # hand check of per-sample D: -.02, -.02, -.18, -.18
    np.testing.assert_array_almost_equal(per[:, 3], [-0.02, -0.02, -0.18, -0.18])
    if reduction == "none":
        np.testing.assert_array_almost_equal(attr, per)
    elif reduction == "sum":
        np.testing.assert_array_almost_equal(attr, per.sum(0))
    else:
        np.testing.assert_array_almost_equal(attr, per.mean(0) + 2 * per.std(0), decimal=5)


@pytest.mark.parametrize("dev", DEVICES)
def test_inplace_relu_eval_module(dev):
    """Gradient capture at an in-place ReLU (the VGG pattern) equals the out-of-place result."""
    d = _dev(dev)
    torch.manual_seed(0)
    base = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(inplace=False),
                         nn.Conv2d(8, 4, 3, padding=1), nn.ReLU(inplace=False), nn.Flatten(), nn.Linear(4 * 36, 5))
    base.eval().to(d)
    inpl = nn.Sequential(*[nn.ReLU(inplace=True) if isinstance(m, nn.ReLU) else m for m in base]).eval().to(d)
    xs = torch.randn(12, 3, 6, 6, device=d)
    ys = torch.randint(0, 5, (12,), device=d)
    dl = DataLoader(TensorDataset(xs, ys), batch_size=4)
    for A in [TaylorAttributionMetric, SensitivityAttributionMetric, APoZAttributionMetric]:
        a1 = A(base, dl, F.cross_entropy, d).run(base[0], find_best_evaluation_module=True)
        a2 = A(inpl, dl, F.cross_entropy, d).run(inpl[0], find_best_evaluation_module=True)
        np.testing.assert_allclose(a1, a2, rtol=1e-5, atol=1e-7)
    # parameters keep requires_grad and get no .grad side effect
    assert all(p.requires_grad for p in base.parameters())


def test_last_path_reports_generic_with_reason():
    """Path transparency: every run records (and logs) which path served it and why the native
    engines were rejected."""
    x, y, model = max_model(torch.device("cpu"))
    m = TaylorAttributionMetric(model, loader(x, y), F.mse_loss, torch.device("cpu"))
    m.run(model[0])
    assert m.last_path["path"] == "generic"
    assert m.last_path["modules"] == ["0"]
    assert any("not a GPU" in r for r in m.last_path["reasons"])
    s = ShapleyAttributionMetric(model, loader(x, y), F.mse_loss, torch.device("cpu"), sv_samples=1)
    s.run(model[0])
    assert s.last_path["path"] == "generic-hook"
