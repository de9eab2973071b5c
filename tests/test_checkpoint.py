"""Pruned-model save/load (shape-restoring) and resumable attribution runs."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import APoZAttributionMetric, Pruner, TaylorAttributionMetric, get_vgg_pruning_graph
from torchpruner_amd.checkpoint import load_pruned, save_pruned
from torchpruner_amd.data import DeviceLoader
from torchpruner_amd.models import vgg_cifar


def test_save_load_pruned_roundtrip(tmp_path):
    torch.manual_seed(0)
    model = vgg_cifar(11).eval()
    x = torch.randn(3, 3, 32, 32)
    pruner = Pruner(model, (3, 32, 32), "cpu")
    rng = np.random.RandomState(0)
    for module, cascade in get_vgg_pruning_graph(model)[:4]:
        n = module.weight.shape[0]
        pruner.prune_model(module, rng.choice(n, n // 3, replace=False), cascade)
    ref = model(x)
    path = str(tmp_path / "pruned.pt")
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    save_pruned(model, path, optimizer=opt)
    fresh = vgg_cifar(11).eval()
    load_pruned(fresh, path)
    torch.testing.assert_close(fresh(x), ref)
    assert fresh.classifier[0].p == model.classifier[0].p  # Dropout rate adjusted by the cascade
    assert [m.out_channels for m in fresh.features if isinstance(m, nn.Conv2d)] == \
        [m.out_channels for m in model.features if isinstance(m, nn.Conv2d)]


class Interrupting:
    """Loader that raises after ``stop`` batches on its first pass (simulated failure)."""

    def __init__(self, loader, stop):
        self.loader, self.stop, self.armed = loader, stop, True
        self.dataset = loader.dataset

    def __iter__(self):
        for i, b in enumerate(self.loader):
            if self.armed and i == self.stop:
                self.armed = False
                raise RuntimeError("simulated failure")
            yield b


@pytest.mark.parametrize("metric", [TaylorAttributionMetric, APoZAttributionMetric])
@pytest.mark.parametrize("reduction", ["mean", "none"])
def test_resume_after_failure(tmp_path, metric, reduction):
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(6, 8), nn.ReLU(), nn.Linear(8, 3)).eval()
    x, y = torch.randn(40, 6), torch.randint(0, 3, (40,))
    dl = DeviceLoader(x, y, 4)
    ref = metric(model, dl, F.cross_entropy, "cpu", reduction=reduction).run(model[0])
    flaky = Interrupting(dl, stop=6)
    ck = str(tmp_path / "attr.ckpt")
    m = metric(model, flaky, F.cross_entropy, "cpu", reduction=reduction, checkpoint=ck, checkpoint_every=2)
    with pytest.raises(RuntimeError):
        m.run(model[0])
    got = m.run(model[0])  # resumes from the last checkpoint, recomputes only the rest
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)
