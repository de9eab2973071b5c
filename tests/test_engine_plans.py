"""CPU checks of the engines' lowering decisions (no GPU needed): which models/modules the fused
VGG chain, the ResNet engine and the native training path accept, and channel padding."""
import numpy as np
import torch
import torch.nn as nn

from torchpruner_amd import Pruner, get_resnet_pruning_graph


def test_cpad():
    from torchpruner_amd.engine.fused_chain import cpad
    assert [cpad(c) for c in (1, 31, 32, 33, 64, 100)] == [32, 32, 32, 64, 64, 128]
    assert cpad(5, 4) == 8


def test_resnet_plan_accepts_pruned_widths():
    from torchpruner_amd.engine.resnet_engine import build_resnet_plan
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, width=32).eval()
    rng = np.random.RandomState(0)
    pruner = Pruner(model, (3, 32, 32), "cpu")
    for module, cascade in get_resnet_pruning_graph(model):
        n = module.weight.shape[0]
        pruner.prune_model(module, rng.choice(n, 7, replace=False), cascade)
    plan, why = build_resnet_plan(model)
    assert plan is not None, why
    assert any(c.conv.out_channels % 32 for b in plan.blocks for c in b.convs)


def test_resnet_plan_rejects_non_resnets():
    from torchpruner_amd.engine.resnet_engine import build_resnet_plan
    from torchpruner_amd.models import prunable_vgg16
    plan, why = build_resnet_plan(prunable_vgg16())
    assert plan is None and "ResNet" in why


def test_native_training_eligibility():
    from torchpruner_amd.engine.train import eligible
    assert eligible(nn.Conv2d(16, 32, 3, padding=1))
    assert eligible(nn.Conv2d(64, 128, 1, stride=2))
    assert eligible(nn.Conv2d(3, 64, 7, stride=2, padding=3))
    assert eligible(nn.Conv2d(16, 32, 5, padding=2))              # 5x5 (FMNIST conv1)
    assert eligible(nn.Conv2d(1, 32, 5, padding=2))               # tiny-Cin packed taps
    assert eligible(nn.Conv2d(32, 64, 3, padding=2))              # FMNIST conv2: pad 2
    assert not eligible(nn.Conv2d(16, 32, 5, stride=2, padding=2))  # no strided 5x5 dgrad
    assert not eligible(nn.Conv2d(16, 32, 3, padding=3))          # pad > ks - 1
    assert not eligible(nn.Conv2d(16, 32, 3, groups=2))           # grouped
    assert not eligible(nn.Conv2d(16, 32, 3, dilation=2))         # dilated
    assert not eligible(nn.Conv2d(16, 32, (1, 3)))                # non-square
    assert not eligible(nn.Conv2d(16, 32, 3, padding="same"))     # string padding
    assert not eligible(nn.Conv2d(16, 32, 3, padding=1, padding_mode="reflect"))
    assert not eligible(nn.Linear(4, 4))


def test_native_convs_is_a_noop_without_gpu_kernels(monkeypatch):
    """On CPU (or with TORCHPRUNER_BACKEND=torch) nothing is switched and modules are untouched."""
    from torchpruner_amd.engine.train import native_convs
    monkeypatch.setenv("TORCHPRUNER_BACKEND", "torch")
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU())
    with native_convs(model) as switched:
        assert switched == []
        y = model(torch.randn(2, 3, 8, 8))
    assert y.shape == (2, 8, 8, 8)
    assert all("forward" not in m.__dict__ for m in model.modules())


def test_debug_sync_proxy_wraps_ops(monkeypatch):
    from torchpruner_amd.ops import _native
    monkeypatch.setenv("TORCHPRUNER_DEBUG_SYNC", "1")

    class _NS:
        @staticmethod
        def add_one(x):
            return x + 1

    synced = []
    monkeypatch.setattr(torch.cuda, "synchronize", lambda: synced.append(1))
    proxy = _native._SyncOps(_NS())
    assert proxy.add_one(1) == 2 and synced == [1]


def test_reference_module_paths_import():
    """Code importing the reference's submodules (not just the packages) runs unchanged."""
    import importlib
    import torchpruner_amd as tp
    paths = {
        "torchpruner.attributions.attributions": ["_AttributionMetric", "SUPPORTED_OUT_PRUNING_MODULES"],
        "torchpruner.attributions.methods.random": ["RandomAttributionMetric"],
        "torchpruner.attributions.methods.weight_norm": ["WeightNormAttributionMetric"],
        "torchpruner.attributions.methods.apoz": ["APoZAttributionMetric"],
        "torchpruner.attributions.methods.sensitivity": ["SensitivityAttributionMetric"],
        "torchpruner.attributions.methods.taylor": ["TaylorAttributionMetric"],
        "torchpruner.attributions.methods.shapley_values": ["ShapleyAttributionMetric"],
        "torchpruner.pruner.pruner": ["Pruner", "SUPPORTED_IN_PRUNING_MODULES"],
        "torchpruner.pruner.opt_pruner": ["OptimizerPruner"],
        "torchpruner.utils.graph": ["find_best_module_for_attributions", "get_vgg_pruning_graph", "ACTIVATIONS"],
    }
    for mod, names in paths.items():
        m = importlib.import_module(mod)
        for n in names:
            obj = getattr(m, n)
            if hasattr(tp, n):
                assert obj is getattr(tp, n), (mod, n)


def test_prefetch_cpu_passthrough():
    from torchpruner_amd.data import prefetch_to_device
    items = [(i, torch.full((2,), float(i))) for i in range(5)]
    out = list(prefetch_to_device(items, "cpu"))
    assert [o[0] for o in out] == list(range(5)) and all(o[1][0] == i for i, o in enumerate(out))


import pytest  # noqa: E402


@pytest.mark.gpu
def test_prefetch_host_loader_matches_device_loader(cuda):
    """A CPU DataLoader (pinned + copied ahead on a side stream) gives the same scores as
    device-resident batches, in the same order."""
    import torch.nn.functional as F
    from torch.utils.data import DataLoader, TensorDataset
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader, prefetch_to_device
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    x, y = torch.randn(40, 3, 32, 32), torch.randint(0, 10, (40,))
    convs = [m for m in model.features if isinstance(m, nn.Conv2d)][:4]
    host = DataLoader(TensorDataset(x, y), batch_size=8, shuffle=False)
    a = TaylorAttributionMetric(model, host, F.cross_entropy, cuda, reduction="none").run_many(convs, True)
    b = TaylorAttributionMetric(model, DeviceLoader(x.to(cuda), y.to(cuda), 8), F.cross_entropy, cuda,
                                reduction="none").run_many(convs, True)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)
    got = [int(t[1][0]) for t in prefetch_to_device(((i, torch.full((3,), i)) for i in range(7)), cuda, depth=3)]
    assert got == list(range(7))


class _TinyRes(nn.Module):
    """Residual model without forward_partial: Shapley's slow (hook) path."""

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(6, 8)
        self.fc2 = nn.Linear(8, 6)
        self.head = nn.Linear(6, 3)

    def forward(self, x):
        h = torch.relu(self.fc1(x))
        return self.head(torch.relu(self.fc2(h) + x))


def test_shapley_slow_path_batched_prefixes_on_residual_model():
    import torch.nn.functional as F
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    torch.manual_seed(0)
    model = _TinyRes().eval()
    x, y = torch.randn(10, 6), torch.randint(0, 3, (10,))
    out = []
    for pb in (1, None):  # one prefix per forward vs K stacked prefixes per forward
        np.random.seed(3)
        out.append(ShapleyAttributionMetric(model, DeviceLoader(x, y, 5), F.cross_entropy, "cpu", sv_samples=3,
                                            prefix_batch=pb).run(model.fc1))
    np.testing.assert_allclose(out[0], out[1], rtol=1e-5, atol=1e-7)
