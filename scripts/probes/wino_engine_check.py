"""Engine Taylor scores with the Winograd path on vs off (same model, same batch)."""
import torch

from torchpruner_amd.engine import fused_chain as fc
from torchpruner_amd.models import vgg_cifar

torch.manual_seed(0)
dev = torch.device("cuda")
model = vgg_cifar(16, batch_norm=True).to(dev).eval()
x = torch.randn(256, 3, 32, 32, device=dev)
y = torch.randint(0, 10, (256,), device=dev)
plan, _ = fc.build_plan(model)
res = {}
for wino in (False, True):
    eng = fc.FusedChainEngine(model, plan)
    eng.use_wino = wino
    fc.TUNER.cache.clear()
    out = eng.taylor(x, y)
    res[wino] = {k: v.clone() for k, v in out.items()}
    print("wino", wino, "choices:", sorted(set(v for v in fc.TUNER.cache.values())))
for k in sorted(res[False]):
    a, b = res[False][k].double(), res[True][k].double()
    rel = ((a - b).norm() / a.norm()).item()
    print(f"block {k:2d}: rel diff {rel:.3e}  |a| {a.norm().item():.3e}  |b| {b.norm().item():.3e}")
