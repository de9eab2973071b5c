"""Coalesced small loader batches on the fused engine (attributions/base.py COALESCE_ELEMS): k
consecutive equal-shape batches run as one engine launch with each loader batch's 1/B loss
scaling, so the Taylor / Sensitivity / APoZ scores equal the batch-by-batch ones (up to the
rounding of different kernel choices); leftover and odd-shaped batches run alone."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _loader(x, y, sizes):
    out, o = [], 0
    for s in sizes:
        out.append((x[o:o + s], y[o:o + s]))
        o += s
    return out


@pytest.mark.parametrize("metric", ["taylor", "sensitivity", "apoz"])
def test_coalesced_batches_match_batch_by_batch(cuda, monkeypatch, metric):
    from torchpruner_amd import APoZAttributionMetric, SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.engine.fused_chain import TUNER
    from torchpruner_amd.models import prunable_vgg16
    cls = {"taylor": TaylorAttributionMetric, "sensitivity": SensitivityAttributionMetric,
           "apoz": APoZAttributionMetric}[metric]
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    sizes = [100] * 12 + [37]  # two groups of 5, two leftovers, an odd last batch
    x = torch.randn(sum(sizes), 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (sum(sizes),), device=cuda)
    with TUNER.fixed():
        monkeypatch.setenv("TORCHPRUNER_COALESCE", "0")
        ref_m = cls(model, _loader(x, y, sizes), F.cross_entropy, cuda)
        ref = ref_m.run_many(convs, True)
        assert ref_m.last_coalesce == 1
        monkeypatch.setenv("TORCHPRUNER_COALESCE", "1")
        m = cls(model, _loader(x, y, sizes), F.cross_entropy, cuda)
        got = m.run_many(convs, True)
        assert m.last_path["path"] == "fused" and m.last_coalesce == 5, (m.last_path, m.last_coalesce)
    for k, (a, b) in enumerate(zip(got, ref)):
        # APoZ: exact counts, but a value within an ulp of 0 may round to the other side under
        # another kernel choice
        # Taylor: per-sample sums with cancellation, so a unit's mean can move by ~1e-4 relative
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-5 * np.abs(b).max(), err_msg=str(k))
        assert np.median(np.abs(a - b) / (np.abs(b) + 1e-30)) < 1e-4, k


@pytest.mark.parametrize("metric", ["taylor", "apoz"])
def test_oversized_batch_runs_in_slices(cuda, monkeypatch, metric):
    """A batch over the engine's max_batch (32-bit buffer descriptors) runs in slices with the
    whole batch's loss scaling: same scores as one launch (forced small limit here)."""
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.engine.fused_chain import TUNER, FusedChainEngine
    from torchpruner_amd.models import prunable_vgg16
    cls = TaylorAttributionMetric if metric == "taylor" else APoZAttributionMetric
    torch.manual_seed(3)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(300, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (300,), device=cuda)
    monkeypatch.setenv("TORCHPRUNER_COALESCE", "0")
    with TUNER.fixed():
        ref = cls(model, _loader(x, y, [150, 150]), F.cross_entropy, cuda).run_many(convs, True)
        monkeypatch.setattr(FusedChainEngine, "max_batch", lambda self, shape: 64)
        got = cls(model, _loader(x, y, [150, 150]), F.cross_entropy, cuda).run_many(convs, True)
    for k, (a, b) in enumerate(zip(got, ref)):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-5 * np.abs(b).max(), err_msg=str(k))


@pytest.mark.parametrize("metric", ["taylor", "apoz"])
def test_resnet_oversized_batch_runs_in_slices(cuda, monkeypatch, metric):
    """The ResNet engine passes slice batches past ResNetEngine.max_batch the same way."""
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.engine.fused_chain import TUNER
    from torchpruner_amd.engine.resnet_engine import ResNetEngine
    from torchpruner_amd.models import resnet50
    cls = TaylorAttributionMetric if metric == "taylor" else APoZAttributionMetric
    torch.manual_seed(4)
    model = resnet50(num_classes=10).to(cuda).eval().to(memory_format=torch.channels_last)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    x = torch.randn(40, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (40,), device=cuda)
    with TUNER.fixed():
        m0 = cls(model, _loader(x, y, [20, 20]), F.cross_entropy, cuda)
        ref = m0.run_many(mods, True)
        assert m0.last_path["path"] == "resnet", m0.last_path
        monkeypatch.setattr(ResNetEngine, "max_batch", lambda self, shape: 7)
        m1 = cls(model, _loader(x, y, [20, 20]), F.cross_entropy, cuda)
        got = m1.run_many(mods, True)
        assert m1.last_path["path"] == "resnet", m1.last_path
    for k, (a, b) in enumerate(zip(got, ref)):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-5 * np.abs(b).max(), err_msg=str(k))
