"""Signed vs unsigned Taylor on the fused VGG engine against the generic path (diagnostic)."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402

cuda = torch.device("cuda")
torch.manual_seed(0)
model = prunable_vgg16().to(cuda).eval()
convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)][:3]
x = torch.randn(48, 3, 32, 32, device=cuda)
y = torch.randint(0, 10, (48,), device=cuda)
dl = DeviceLoader(x, y, 16)
res = {}
for signed in (False, True):
    for be in ("hip", "torch"):
        os.environ["TORCHPRUNER_BACKEND"] = be
        m = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda, signed=signed, reduction="none")
        res[(signed, be)] = m.run_many(convs, True)
        print(signed, be, m.last_path["path"])
os.environ.pop("TORCHPRUNER_BACKEND")
for li in range(3):
    fs, fu = res[(True, "hip")][li], res[(False, "hip")][li]
    gs, gu = res[(True, "torch")][li], res[(False, "torch")][li]
    print(f"layer {li}: fused signed==|signed| {np.allclose(fs, np.abs(fs))}  generic signed==|signed| "
          f"{np.allclose(gs, np.abs(gs))}  |fs-gs| {np.abs(fs - gs).max():.2e}  |fu-gu| {np.abs(fu - gu).max():.2e} "
          f"max|gs| {np.abs(gs).max():.2e} min gs {gs.min():.2e} min fs {fs.min():.2e}")
import copy  # noqa: E402
m64 = copy.deepcopy(model).double().cpu()
c64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)][:3]
ex = TaylorAttributionMetric(m64, DeviceLoader(x.double().cpu(), y.cpu(), 16), F.cross_entropy, "cpu", signed=True,
                             reduction="none").run_many(c64, True)
for li in range(3):
    e, fs, gs = ex[li], res[(True, "hip")][li], res[(True, "torch")][li]
    bad_f = np.sign(fs) != np.sign(e)
    bad_g = np.sign(gs) != np.sign(e)
    print(f"layer {li}: sign flips fused {bad_f.sum()} generic {bad_g.sum()} of {e.size}; |fs-e| {np.abs(fs - e).max():.2e}"
          f" |gs-e| {np.abs(gs - e).max():.2e}; worst fused entry e={e.flat[np.abs(fs - e).argmax()]:.3e} "
          f"fs={fs.flat[np.abs(fs - e).argmax()]:.3e} gs={gs.flat[np.abs(fs - e).argmax()]:.3e}")
