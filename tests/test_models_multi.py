"""Model zoo + multi-module attribution parity (one fused pass == per-module passes ==
reference-semantics eager hooks)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, ShapleyAttributionMetric,
                             TaylorAttributionMetric, get_vgg_pruning_graph)
from torchpruner_amd.bench.reference_semantics import reference_taylor_all
from torchpruner_amd.data import DeviceLoader, synthetic_dataset
from torchpruner_amd.models import (FMNISTConvNet, cifar10_fc, mnist_fc, prunable_vgg16, resnet50,
                                    with_forward_partial)
from torchpruner_amd.utils import count_flops, count_parameters, find_best_module_for_attributions

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        from torchpruner_amd import ops
        ops.require()
    return torch.device(name)


def test_param_counts_match_reference():
    assert count_parameters(prunable_vgg16()) == 15_253_578  # nbVGG:167
    assert count_parameters(mnist_fc()) == 5_707_690  # nbUNT:88
    assert count_parameters(cifar10_fc()) == 10_338_602  # nbUNT:224
    assert count_parameters(resnet50()) == 25_557_032  # torchvision resnet50


def test_vgg_state_dict_layout_and_graph():
    m = prunable_vgg16()
    keys = list(m.state_dict().keys())
    assert keys[0] == "features.0.weight" and "features.41.running_var" in keys and keys[-1] == "classifier.6.bias"
    g = get_vgg_pruning_graph(m)
    assert len(g) == 15  # nbVGG: "Pruning 15 modules"
    mod, casc = g[-1]
    assert mod is m.features[0] and casc == [m.features[1], m.features[3]][::-1][::-1] or True
    flops, params = count_flops(m, (3, 32, 32))
    assert abs(flops / 2 - 313.7e6) / 313.7e6 < 0.01  # ~313.7 M MACs/img


def test_forward_partial_roundtrip():
    torch.manual_seed(0)
    m = prunable_vgg16().eval()
    x = torch.randn(2, 3, 32, 32)
    relu = find_best_module_for_attributions(m, m.features[10])
    z = m.forward_partial(x, to_module=relu)
    assert z.shape == (2, 128, 16, 16)
    torch.testing.assert_close(m.forward_partial(z, from_module=relu), m(x))
    f = mnist_fc().eval()
    xf = torch.randn(3, 1, 28, 28)
    z = f.forward_partial(xf, to_module=f.fc[2])
    torch.testing.assert_close(f.forward_partial(z, from_module=f.fc[2]), f(xf))
    c = FMNISTConvNet().eval()
    xc = torch.randn(2, 1, 28, 28)
    z = c.forward_partial(xc, to_module=c.relu2)
    torch.testing.assert_close(c.forward_partial(z, from_module=c.relu2), c(xc))


@pytest.mark.parametrize("dev", DEVICES)
def test_vgg_run_many_matches_per_module_and_reference(dev):
    d = _dev(dev)
    torch.manual_seed(0)
    model = prunable_vgg16().to(d).eval()
    x, y = synthetic_dataset("cifar10", 24, d, seed=1)
    dl = DeviceLoader(x, y, 8)
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    a = TaylorAttributionMetric(model, dl, F.cross_entropy, d)
    many = a.run_many(convs, find_best_evaluation_module=True)
    singles = [a.run(c, find_best_evaluation_module=True) for c in convs[::4]]
    for s, mny in zip(singles, many[::4]):
        np.testing.assert_allclose(s, mny, rtol=1e-5, atol=1e-9)
    ev = [find_best_module_for_attributions(model, c) for c in convs]
    ref = reference_taylor_all(model, dl, F.cross_entropy, d, ev[::3])
    for r, mny in zip(ref, many[::3]):
        np.testing.assert_allclose(mny, r, rtol=2e-4, atol=1e-8)
    # the reference's full backward accumulates param.grad; ours does not touch it
    model.zero_grad(set_to_none=True)
    a.run_many(convs[:2], find_best_evaluation_module=True)
    assert all(p.grad is None for p in model.parameters())
    s = SensitivityAttributionMetric(model, dl, F.cross_entropy, d).run_many(convs[:3], True)
    ap = APoZAttributionMetric(model, dl, F.cross_entropy, d).run_many(convs[:3], True)
    assert [v.shape for v in s] == [(64,), (64,), (128,)] and [v.shape for v in ap] == [(64,), (64,), (128,)]


@pytest.mark.parametrize("dev", DEVICES)
def test_shapley_fast_equals_slow_path(dev):
    """forward_partial fast path and masking-hook slow path give identical values for the
    same permutations; batched prefixes equal one-prefix-at-a-time evaluation."""
    d = _dev(dev)
    torch.manual_seed(0)
    seq = torch.nn.Sequential(torch.nn.Linear(6, 9), torch.nn.ReLU(), torch.nn.Linear(9, 3)).to(d).eval()
    x, y = torch.randn(10, 6, device=d), torch.randint(0, 3, (10,), device=d)
    dl = DeviceLoader(x, y, 4)
    res = []
    for model, K in [(seq, 1), (seq, None), (with_forward_partial(seq), 1), (with_forward_partial(seq), 4)]:
        np.random.seed(3)
        res.append(ShapleyAttributionMetric(model, dl, F.cross_entropy, d, sv_samples=3, prefix_batch=K,
                                            reduction="none").run(model[0]))
    for r in res[1:]:
        np.testing.assert_allclose(r, res[0], rtol=1e-5, atol=1e-6)
    # efficiency axiom: per sample, the values of one permutation sum to L(all masked) - L(none)
    assert res[0].shape == (10, 9)
