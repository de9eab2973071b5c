"""Is the B=100 fused-engine step host-bound? Times the host side of every pipelined batch
(``_BatchPipeline.take``: Python + kernel launches of one engine forward/backward and its fold)
against the wall time of the whole run, for VGG16-BN Taylor at B=100 (random init, synthetic data).
Usage: python scripts/probes/b100_host_probe.py [--batch 100] [--steps 200]"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.attributions import base  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    B, n = args.batch, args.steps
    x = torch.randn(n * B, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (n * B,), device=dev)
    host = {"t": 0.0, "n": 0}
    orig = base._BatchPipeline.take

    def take(self, *a, **k):
        t0 = time.perf_counter()
        r = orig(self, *a, **k)
        host["t"] += time.perf_counter() - t0
        host["n"] += 1
        return r

    base._BatchPipeline.take = take
    for rep in range(3):
        host.update(t=0.0, n=0)
        m = TaylorAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.run_many(convs, find_best_evaluation_module=True)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"rep {rep}: {n} batches of {B}: wall {wall * 1e3:.1f} ms ({n * B / wall:.0f} img/s); host time in "
              f"pipeline.take {host['t'] * 1e3:.1f} ms over {host['n']} calls "
              f"({host['t'] / max(host['n'], 1) * 1e6:.0f} us/batch vs {wall / n * 1e6:.0f} us/batch wall)",
              flush=True)


if __name__ == "__main__":
    main()
