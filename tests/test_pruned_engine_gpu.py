"""Engines on PRUNED models: odd channel counts (not multiples of 32) are carried zero-padded.

Iterative pruning (score -> prune -> finetune -> score again, nbUNT:169-193) leaves layers with
arbitrary widths; the fused VGG engine and the ResNet engine must keep serving them (instead of
falling back to the generic hook path) and return scores of the REAL width only."""
import copy
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from torchpruner_amd import Pruner, get_resnet_pruning_graph, get_vgg_pruning_graph


def _prune_vgg_odd(model, device, seed=0):
    rng = np.random.RandomState(seed)
    pruner = Pruner(model, (3, 32, 32), device)
    for module, cascade in get_vgg_pruning_graph(model):
        n = module.weight.shape[0]
        k = int(rng.randint(1, max(2, n // 3)))  # 1 .. n/3 units -> odd widths
        pruner.prune_model(module, rng.choice(n, k, replace=False), cascading_modules=cascade)
    return model


def test_vgg_plan_pads_pruned_widths():
    from torchpruner_amd.engine.fused_chain import build_plan, cpad
    from torchpruner_amd.models import prunable_vgg16
    model = _prune_vgg_odd(prunable_vgg16().eval(), "cpu")
    plan, why = build_plan(model)
    assert plan is not None, why
    widths = [b.conv.out_channels for b in plan.convs]
    assert any(w % 32 for w in widths)
    for b in plan.convs[1:]:
        assert b.width == cpad(b.conv.out_channels)
    assert plan.linears[-1].width == plan.linears[-1].linear.out_features


def _bn_stats(model):
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)


@pytest.mark.gpu
def test_pruned_vgg_engine_taylor_matches_fp64(cuda):
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(0)
    model = _prune_vgg_odd(prunable_vgg16().to(cuda).eval(), cuda)
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    lins = [model.classifier[1], model.classifier[4]]
    ev = [find_best_module_for_attributions(model, m) for m in convs + lins]
    assert maybe_engine(model, ev, F.cross_entropy, cuda) is not None
    x = torch.randn(32, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (32,), device=cuda)
    dl = DeviceLoader(x, y, 16)
    m64 = copy.deepcopy(model).double().cpu()
    c64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)] + [m64.classifier[1], m64.classifier[4]]
    dl64 = DeviceLoader(x.double().cpu(), y.cpu(), 16)
    for red in ("mean", "none"):
        fused = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda, reduction=red).run_many(convs + lins, True)
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            exact = TaylorAttributionMetric(m64, dl64, F.cross_entropy, "cpu", reduction=red).run_many(c64, True)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
        for mod, a, e in zip(convs + lins, fused, exact):
            assert a.shape == e.shape and a.shape[-1] == mod.weight.shape[0]
            err = np.abs(a - e).max() / (np.abs(e).max() + 1e-30)
            assert err < (5e-3 if red == "mean" else 2e-2), (mod, err)


@pytest.mark.gpu
@pytest.mark.parametrize("layer", [2, 9, 13])
def test_pruned_vgg_engine_shapley_and_ablation(cuda, layer):
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    from torchpruner_amd.utils.ablation import ablation_curve
    torch.manual_seed(1)
    model = _prune_vgg_odd(prunable_vgg16().to(cuda).eval(), cuda, seed=1)
    prunable = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1],
                                                                                 model.classifier[4]]
    module = prunable[layer]
    x = torch.randn(8, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    m64 = copy.deepcopy(model).double().cpu()
    p64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)] + [m64.classifier[1], m64.classifier[4]]
    from torchpruner_amd.engine.fused_chain import TUNER
    res = []
    for backend, mdl, mod, d, xx, yy in (("hip", model, module, cuda, x, y), ("torch", model, module, cuda, x, y),
                                         ("torch", m64, p64[layer], "cpu", x.double().cpu(), y.cpu())):
        os.environ["TORCHPRUNER_BACKEND"] = backend
        try:
            np.random.seed(5)
            with TUNER.fixed():  # pinned kernel choices: the fused numbers are the same on any box
                res.append(ShapleyAttributionMetric(mdl, DeviceLoader(xx, yy, 4), F.cross_entropy, d,
                                                    sv_samples=2).run(mod, find_best_evaluation_module=True))
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
    assert res[0].shape == (module.weight.shape[0],)
    # single-unit deltas of a random-init net sit near fp32 loss rounding: bound the error in fp32
    # ulps of the mean loss (forward-only values: no dependence on another library's algorithm)
    with torch.no_grad():
        lbar = float(F.cross_entropy(m64(x.double().cpu()), y.cpu()))
    err_fused, err_generic = np.abs(res[0] - res[2]).max(), np.abs(res[1] - res[2]).max()
    ulps = err_fused / (np.finfo(np.float32).eps * lbar)
    print(f"pruned layer {layer}: fused_err={err_fused:.2e} ({ulps:.0f} ulps) miopen_err={err_generic:.2e}")
    assert ulps < 100, (err_fused, err_generic, lbar)
    ev = find_best_module_for_attributions(model, module)
    ranking = np.random.RandomState(0).permutation(module.weight.shape[0])
    l_hip, a_hip = ablation_curve(model, ev, ranking, x, y)
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        l_ref, a_ref = ablation_curve(model, ev, ranking, x, y)
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]
    assert len(l_hip) == module.weight.shape[0] + 1
    np.testing.assert_allclose(l_hip, l_ref, rtol=2e-3, atol=2e-4)


@pytest.mark.gpu
def test_pruned_resnet_engine_apoz_matches_generic(cuda):
    from torchpruner_amd import APoZAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_resnet_engine
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 2, 1, 1], num_classes=10, width=32).to(cuda).eval()
    _bn_stats(model)
    pruner = Pruner(model, (3, 64, 64), cuda)
    rng = np.random.RandomState(0)
    for module, cascade in get_resnet_pruning_graph(model):
        n = module.weight.shape[0]
        pruner.prune_model(module, rng.choice(n, int(n * 0.3) + 1, replace=False), cascade)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    assert any(m.weight.shape[0] % 32 for m in mods)
    ev = [find_best_module_for_attributions(model, m) for m in mods]
    eng = maybe_resnet_engine(model, ev, cuda)
    assert eng is not None
    x = torch.randn(8, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    dl = DeviceLoader(x, y, 4)
    fused = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(mods, True)
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        generic = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(mods, True)
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]
    for m, a, b in zip(mods, fused, generic):
        assert a.shape == b.shape == (m.weight.shape[0],)
        np.testing.assert_allclose(a, b, atol=0.5)
    with torch.no_grad():
        torch.testing.assert_close(eng.forward(x), model(x), rtol=2e-3, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("prune", [False, True])
def test_vgg_engine_sensitivity_matches_fp64(cuda, prune):
    """Sensitivity (sum |dL/da|) from the fused dgrad epilogues vs an fp64 oracle."""
    from torchpruner_amd import SensitivityAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(2)
    model = prunable_vgg16().to(cuda).eval()
    if prune:
        _prune_vgg_odd(model, cuda, seed=2)
    mods = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1], model.classifier[4]]
    assert maybe_engine(model, [find_best_module_for_attributions(model, m) for m in mods], F.cross_entropy,
                        cuda) is not None
    x = torch.randn(32, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (32,), device=cuda)
    m64 = copy.deepcopy(model).double().cpu()
    mods64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)] + [m64.classifier[1], m64.classifier[4]]
    for red in ("mean", "none"):
        got = SensitivityAttributionMetric(model, DeviceLoader(x, y, 16), F.cross_entropy, cuda,
                                           reduction=red).run_many(mods, True)
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            ref = SensitivityAttributionMetric(m64, DeviceLoader(x.double().cpu(), y.cpu(), 16), F.cross_entropy,
                                               "cpu", reduction=red).run_many(mods64, True)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
        for m, a, r in zip(mods, got, ref):
            assert a.shape == r.shape and a.shape[-1] == m.weight.shape[0]
            e = np.abs(a - r) / (np.abs(r).max() + 1e-30)
            if red == "mean":
                assert e.max() < 5e-3, (m, red, e.max())
            else:  # per-sample sums: a ReLU decision flip (fp32 vs fp64, tuner-chosen kernel) moves one
                # sample's sum by a few %; the bulk must still agree to fp32 accuracy
                assert e.max() < 5e-2 and np.median(e) < 1e-3, (m, red, e.max(), np.median(e))


@pytest.mark.gpu
@pytest.mark.parametrize("prune", [False, True])
def test_vgg_engine_apoz_matches_generic(cuda, prune):
    """APoZ counts fused into the VGG engine's forward epilogues (pre-pool ReLU outputs; Winograd
    / implicit-GEMM / dense-2x2 / classifier blocks) vs the generic hook path."""
    from torchpruner_amd import APoZAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(3)
    model = prunable_vgg16().to(cuda).eval()
    _bn_stats(model)
    if prune:
        _prune_vgg_odd(model, cuda, seed=3)
    mods = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1], model.classifier[4]]
    ev = [find_best_module_for_attributions(model, m) for m in mods]
    assert maybe_engine(model, ev, torch.nn.functional.mse_loss, cuda, need_ce=False) is not None
    x = torch.randn(24, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (24,), device=cuda)
    for red in ("mean", "none"):
        dl = DeviceLoader(x, y, 8)
        got = APoZAttributionMetric(model, dl, F.cross_entropy, cuda, reduction=red).run_many(mods, True)
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            ref = APoZAttributionMetric(model, dl, F.cross_entropy, cuda, reduction=red).run_many(mods, True)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
        for m, a, r in zip(mods, got, ref):
            assert a.shape == r.shape and a.shape[-1] == m.weight.shape[0]
            # exact counts; only outputs within rounding of 0 may flip between the two conv paths
            tol = 0.05 * (r.max() + 1) if red == "mean" else 2.0
            assert np.abs(a - r).max() <= tol, (m, red, np.abs(a - r).max())


@pytest.mark.gpu
@pytest.mark.parametrize("depth,bn", [(11, True), (13, False), (19, True)])
def test_vgg_variants_on_engine(cuda, depth, bn):
    """Every VGG of the zoo (11-19 layers, with / without BN; VGG11 pools right after its
    tiny-Cin first conv) lowers to the fused engine: Taylor vs the fp64 oracle, APoZ vs the
    generic hook path."""
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models.vgg import vgg_cifar
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(depth)
    model = vgg_cifar(depth, batch_norm=bn).to(cuda).eval()
    _bn_stats(model)
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    ev = [find_best_module_for_attributions(model, m) for m in convs]
    assert maybe_engine(model, ev, F.cross_entropy, cuda) is not None
    x = torch.randn(16, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (16,), device=cuda)
    dl = DeviceLoader(x, y, 8)
    got = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(convs, True)
    apoz = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(convs, True)
    m64 = copy.deepcopy(model).double().cpu()
    c64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)]
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        ref = TaylorAttributionMetric(m64, DeviceLoader(x.double().cpu(), y.cpu(), 8), F.cross_entropy,
                                      "cpu").run_many(c64, True)
        apoz_ref = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(convs, True)
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]
    for m, a, r in zip(convs, got, ref):
        assert a.shape == r.shape
        assert np.abs(a - r).max() / (np.abs(r).max() + 1e-30) < 5e-3, m
    for m, a, r in zip(convs, apoz, apoz_ref):
        assert np.abs(a - r).max() <= 0.05 * (r.max() + 1), m
