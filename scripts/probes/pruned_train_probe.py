"""Probe: ResNet-50 training step (224 px, fp32, native kernels, torch fused SGD) dense vs pruned
like config #5 (1 and 2 rounds of 20 % of every prunable bottleneck conv, random indices): the
time per step and the conv MAC ratio of each model, to check that pruned widths turn into speed
(round 1 >= 1.20x dense, round 2 >= 1.45x).

    python scripts/probes/pruned_train_probe.py [--rounds 0,1,2] [--batch 128] [--steps 10]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torchpruner_amd import Pruner, get_resnet_pruning_graph  # noqa: E402
from torchpruner_amd.engine.train import enable_native_convs  # noqa: E402
from torchpruner_amd.models import resnet50  # noqa: E402


def conv_macs(model, res):
    macs = []

    def hook(m, i, o):
        macs.append(o.numel() // o.shape[0] * m.in_channels * m.kernel_size[0] * m.kernel_size[1])
    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, torch.nn.Conv2d)]
    with torch.no_grad():
        model.eval()(torch.zeros(1, 3, res, res, device=next(model.parameters()).device))
    for h in hs:
        h.remove()
    return sum(macs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", default="0,1,2")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--res", type=int, default=224)
    a = ap.parse_args()
    dev = torch.device("cuda")
    dense_ms = None
    for rounds in [int(r) for r in a.rounds.split(",")]:
        torch.manual_seed(0)
        model = resnet50().to(dev)
        rng = np.random.RandomState(0)
        pruner = Pruner(model, (3, a.res, a.res), dev)
        for _ in range(rounds):
            for module, cascade in get_resnet_pruning_graph(model):
                n = module.weight.shape[0]
                pruner.prune_model(module, rng.choice(n, int(n * 0.2), replace=False), cascade)
        macs = conv_macs(model, a.res)
        model = model.to(memory_format=torch.channels_last).train()
        enable_native_convs(model)
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, fused=True)
        x = torch.randn(a.batch, 3, a.res, a.res, device=dev).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (a.batch,), device=dev)

        def step():
            opt.zero_grad(set_to_none=True)
            F.cross_entropy(model(x), y).backward()
            opt.step()

        t = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        warm = time.perf_counter() - t
        t = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        if rounds == 0:
            dense_ms, dense_macs = ms, macs
        widths = sorted({m.out_channels for m in model.modules() if isinstance(m, torch.nn.Conv2d)})
        rel = f", {dense_ms / ms:.3f}x dense for {macs / dense_macs:.3f}x the conv MACs" if dense_ms else ""
        print(f"[pruned_train] rounds={rounds} B={a.batch}: {ms:.2f} ms/step -> {a.batch / ms * 1e3:.0f} img/s"
              f"{rel} (warm-up {warm:.1f}s; widths {widths[:6]}...)", flush=True)
        del model, opt, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
