"""Conv-less chains (the reference's MNIST / CIFAR FC nets, experiments/models/mnist.py:9-35,
cifar10.py:10-36: Flatten -> Linear -> LeakyReLU -> ... -> Linear) on the fused engine: MFMA
GEMMs with NaN-propagating LeakyReLU epilogues and leaky dgrad masks, against an fp64 CPU
oracle of the generic path. Also the CPU lowering decisions for such chains."""
import copy
import os

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


def _fcnet(in_features=784, hidden=200, odd=False):
    from torchpruner_amd.models import FCNet
    torch.manual_seed(0)
    m = FCNet(in_features, hidden=hidden)
    if odd:  # pruned-like widths: not multiples of 32 anywhere
        from torchpruner_amd import Pruner
        layers = list(m.fc.children())
        p = Pruner(m, (in_features,), "cpu")
        p.prune_model(layers[3], [0, 5, 9], [layers[5]])
        p.prune_model(layers[1], [1, 2], [layers[3]])
    return m.eval()


def test_mlp_plan_lowering():
    from torchpruner_amd.engine.fused_chain import build_plan
    plan, why = build_plan(_fcnet())
    assert plan is not None, why
    assert not plan.convs and len(plan.linears) == 3
    assert [b.slope for b in plan.linears[:-1]] == [0.01, 0.01]
    assert plan.linears[0].width == 224 and plan.linears[-1].width == 10
    # an activation with a negative slope is not a block activation
    bad = nn.Sequential(nn.Flatten(), nn.Linear(8, 8), nn.LeakyReLU(-0.5), nn.Linear(8, 2))
    plan, why = build_plan(bad)
    assert plan is None


def _oracle(metric_cls, model, x, y, mods, **kw):
    m64 = copy.deepcopy(model).double().cpu()
    names = {id(m): n for n, m in model.named_modules()}
    mods64 = [dict(m64.named_modules())[names[id(m)]] for m in mods]
    from torchpruner_amd.data import DeviceLoader
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        return metric_cls(m64, DeviceLoader(x.double().cpu(), y.cpu(), 16), F.cross_entropy, "cpu",
                          **kw).run_many(mods64, True)
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]


@pytest.mark.gpu
@pytest.mark.parametrize("odd", [False, True])
def test_mlp_engine_gradient_metrics_match_fp64(cuda, odd):
    from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    model = _fcnet(odd=odd).to(cuda)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(40, 1, 28, 28, generator=g).to(cuda)
    y = torch.randint(0, 10, (40,), generator=g).to(cuda)
    lins = [model.fc[1], model.fc[3]]
    for cls, kw in ((TaylorAttributionMetric, {}), (TaylorAttributionMetric, {"signed": True}),
                    (SensitivityAttributionMetric, {})):
        for red in ("mean", "none"):
            m = cls(model, DeviceLoader(x, y, 16), F.cross_entropy, cuda, reduction=red, **kw)
            got = m.run_many(lins, True)
            assert m.last_path["path"] == "fused", m.last_path
            ref = _oracle(cls, model, x, y, lins, reduction=red, **kw)
            for a, e in zip(got, ref):
                assert a.shape == e.shape
                err = np.abs(a - e).max() / (np.abs(e).max() + 1e-30)
                assert err < 1e-4, (cls.__name__, kw, red, err)


@pytest.mark.gpu
def test_mlp_engine_apoz_and_shapley_at_linear(cuda):
    """APoZ and Shapley accept the Linear itself (pre-activation) as evaluation module, the
    nbUNT usage (``attribution.run(module)``, nbUNT:185)."""
    from torchpruner_amd import APoZAttributionMetric, ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    model = _fcnet(odd=True).to(cuda)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(24, 784, generator=g).to(cuda)
    y = torch.randint(0, 10, (24,), generator=g).to(cuda)
    lin = model.fc[3]
    res = {}
    for backend in ("hip", "torch"):
        os.environ["TORCHPRUNER_BACKEND"] = backend
        try:
            a = APoZAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, cuda)
            res[("apoz", backend)] = a.run(lin)
            np.random.seed(11)
            s = ShapleyAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, cuda, sv_samples=2)
            res[("sv", backend)] = s.run(lin)
            if backend == "hip":
                assert a.last_path["path"] == "fused" and s.last_path["path"] == "fused", (a.last_path, s.last_path)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
    np.testing.assert_allclose(res[("apoz", "hip")], res[("apoz", "torch")], atol=0.05)  # counts / 24 samples
    np.testing.assert_allclose(res[("sv", "hip")], res[("sv", "torch")], rtol=1e-3, atol=2e-6)


@pytest.mark.gpu
def test_mlp_engine_logits_and_nan_propagation(cuda):
    from torchpruner_amd.engine import maybe_engine
    model = _fcnet(odd=True).to(cuda)
    x = torch.randn(16, 784, device=cuda)
    eng, _ = maybe_engine(model, [model.fc[2]], F.cross_entropy, cuda)
    with torch.no_grad():
        logits, _ = eng.forward(x)
        torch.testing.assert_close(logits, model(x), rtol=1e-4, atol=1e-4)
        x[3, 17] = float("nan")  # the pruner's NaN probe must see NaN reach every unit of sample 3
        h, _ = eng.forward(x, stop_after=0)
    h = h.reshape(16, -1)[:, :model.fc[1].out_features]
    assert torch.isnan(h[3]).all() and not torch.isnan(h[[0, 1, 2, 4]]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["mlp_hidden", "mlp_last", "vgg_conv12", "vgg_fc1"])
def test_shapley_prefix_delta_matches_masked_copies(cuda, where):
    """The prefix-delta GEMM (no masked copies) equals the masked-copy evaluation and the fp64
    generic path up to fp32 rounding, for every Linear-fed evaluation point."""
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    g = torch.Generator().manual_seed(7)
    if where.startswith("mlp"):
        model = _fcnet(odd=True).to(cuda)
        x = torch.randn(20, 784, generator=g)
        module = model.fc[1] if where == "mlp_hidden" else model.fc[3]
    else:
        torch.manual_seed(2)
        model = prunable_vgg16().to(cuda).eval()
        x = torch.randn(12, 3, 32, 32, generator=g)
        module = model.features[40] if where == "vgg_conv12" else model.classifier[1]
    y = torch.randint(0, 10, (x.shape[0],), generator=g)
    res = {}
    for mode, backend, dev in (("delta", "hip", cuda), ("copies", "hip", cuda), ("fp64", "torch", "cpu")):
        mdl = model if mode != "fp64" else copy.deepcopy(model).double().cpu()
        mod = module if mode != "fp64" else dict(mdl.named_modules())[
            {id(m): n for n, m in model.named_modules()}[id(module)]]
        xx = x.to(dev).double() if mode == "fp64" else x.to(dev)
        os.environ["TORCHPRUNER_BACKEND"] = backend
        os.environ["TORCHPRUNER_PREFIX_DELTA"] = "1" if mode == "delta" else "0"
        try:
            np.random.seed(3)
            m = ShapleyAttributionMetric(mdl, DeviceLoader(xx, y.to(dev), 5), F.cross_entropy, dev, sv_samples=2,
                                         prefix_batch=7)
            res[mode] = m.run(mod, find_best_evaluation_module=True)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"], os.environ["TORCHPRUNER_PREFIX_DELTA"]
    err_delta = np.abs(res["delta"] - res["fp64"]).max()
    err_copies = np.abs(res["copies"] - res["fp64"]).max()
    assert res["delta"].shape == res["fp64"].shape
    assert err_delta <= 3 * err_copies + 2e-6, (err_delta, err_copies)


def test_mlp_plan_input_shape_checks():
    """A plain Linear chain given a (B, T, F) batch runs per token in PyTorch; the engine would
    read it as one flat vector, so such inputs reject the plan (CPU: lowering decision only)."""
    from torchpruner_amd.engine.fused_chain import build_plan
    plain, _ = build_plan(nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 4)))
    assert plain is not None and not plain.flatten
    assert plain.input_error((5, 8)) is None
    assert plain.input_error((5, 3, 8)) is not None  # per-token in PyTorch
    assert plain.input_error((5, 9)) is not None
    flat, _ = build_plan(_fcnet(in_features=784, hidden=64))
    assert flat.flatten and flat.input_error((5, 1, 28, 28)) is None
    assert flat.input_error((5, 1, 28, 29)) is not None  # wider than in_features
    from torchpruner_amd.models import prunable_vgg16
    vgg, _ = build_plan(prunable_vgg16().eval())
    assert vgg.input_error((2, 3, 32, 32)) is None
    assert vgg.input_error((2, 3, 64, 64)) is not None  # features would not end at 1x1


@pytest.mark.gpu
def test_mlp_engine_rejects_per_token_input(cuda):
    """(B, T, F) input to Sequential(Linear, ReLU, Linear): the metrics take the generic path and
    agree with an fp64 CPU run; native_logits declines."""
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.engine import native_logits
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 4)).eval()
    x = torch.randn(12, 3, 8)
    y = torch.randint(0, 4, (12, 3))

    def crit(out, t, reduction="mean"):
        return F.cross_entropy(out.reshape(-1, 4), t.reshape(-1), reduction=reduction)

    md = copy.deepcopy(m).to(cuda)
    assert native_logits(md, x.to(cuda)) is None
    dl = [(x[i:i + 4].to(cuda), y[i:i + 4].to(cuda)) for i in range(0, 12, 4)]
    for M in (TaylorAttributionMetric, APoZAttributionMetric):
        met = M(md, dl, crit, cuda)
        got = met.run(md[0], find_best_evaluation_module=True)
        assert met.last_path["path"] == "generic", met.last_path
        mc = copy.deepcopy(m).double()
        ref = M(mc, [(a.double(), b) for a, b in zip(x.split(4), y.split(4))], crit, torch.device("cpu")).run(
            mc[0], find_best_evaluation_module=True)
        assert got.shape == ref.shape == (3,)  # units along dim 1 (T), as the reference's hooks reduce
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-6)
