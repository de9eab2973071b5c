"""Does an optimizer step bump the parameters' autograd version counters (the training pack
cache's staleness signal)? And does native-conv training with the batched weight-pack cache
follow the per-call packing loss trajectory? python scripts/probes/pack_cache_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

for kind in ("foreach", "fused"):
    p = torch.nn.Parameter(torch.randn(64, 64, 3, 3, device="cuda"))
    opt = torch.optim.SGD([p], lr=0.1, momentum=0.9, weight_decay=1e-4, **{kind: True})
    p.grad = torch.randn_like(p)
    v0 = p._version
    opt.step()
    print(f"{kind} SGD: version {v0} -> {p._version}", flush=True)

from torchpruner_amd.engine import train as tr  # noqa: E402
from torchpruner_amd.models import resnet18  # noqa: E402

for batch_pack in (False, True):
    for kind in ("foreach", "fused"):
        tr._BATCH_PACK = batch_pack
        torch.manual_seed(0)
        m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
        tr.enable_native_convs(m)
        opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, **{kind: True})
        x = torch.randn(32, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (32,), device="cuda")
        losses = []
        for _ in range(15):
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            losses.append(round(loss.item(), 4))
        print(f"batch_pack={batch_pack} {kind}: {losses}", flush=True)
