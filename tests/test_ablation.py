"""Batched ablation curve == the notebook's sequential index_fill_ loop (nbVGG:1270-1282)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from torchpruner_amd.models import prunable_vgg16, mnist_fc
from torchpruner_amd.utils import find_best_module_for_attributions
from torchpruner_amd.utils.ablation import ablation_auc, ablation_curve

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _sequential(model, ev, ranking, x, y):
    z = model.forward_partial(x, to_module=ev)
    out = model.forward_partial(z, from_module=ev)
    losses = [float(F.cross_entropy(out, y))]
    accs = [float((out.argmax(1) == y).float().mean())]
    for i in ranking:
        z.index_fill_(1, torch.tensor([int(i)], device=x.device), 0.0)
        out = model.forward_partial(z, from_module=ev)
        losses.append(float(F.cross_entropy(out, y)))
        accs.append(float((out.argmax(1) == y).float().mean()))
    return np.array(losses), np.array(accs)


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("which", ["vgg_conv", "vgg_fc", "mlp"])
def test_ablation_matches_sequential(dev, which):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = torch.device(dev)
    torch.manual_seed(0)
    if which == "mlp":
        model = mnist_fc().to(d).eval()
        module = model.fc[3]
        x = torch.randn(20, 1, 28, 28, device=d)
    else:
        model = prunable_vgg16().to(d).eval()
        module = model.features[40] if which == "vgg_conv" else model.classifier[4]
        x = torch.randn(20, 3, 32, 32, device=d)
    y = torch.randint(0, 10, (20,), device=d)
    ev = find_best_module_for_attributions(model, module)
    n = module.out_channels if hasattr(module, "out_channels") else module.out_features
    ranking = np.random.RandomState(0).permutation(n)[:40]
    with torch.no_grad():
        ls, acs = _sequential(model, ev, ranking, x, y)
        lb, ab = ablation_curve(model, ev, ranking, x, y, max_eval_elements=1 << 16)
    np.testing.assert_allclose(lb[: len(ls)], ls, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(ab[: len(acs)], acs)
    assert ablation_auc([1.0, 1.5, 2.0]) == pytest.approx(0.75)
