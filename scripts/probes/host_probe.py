"""Host-boundness of an attribution run: the host time until the run's first score
finalisation (everything enqueued, nothing waited for) against the run's wall time. A ratio
near 1 means the GPU waits for Python; well below 1 means the run is GPU-bound.

    python scripts/probes/host_probe.py shapley --layer 6      # VGG16 Shapley S=5, 1000 images, B=100
    python scripts/probes/host_probe.py taylor --batch 100     # VGG16 Taylor, 200 batches
    python scripts/probes/host_probe.py resnet-taylor --batch 256
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import (APoZAttributionMetric, ShapleyAttributionMetric,  # noqa: E402
                             TaylorAttributionMetric)
from torchpruner_amd.attributions import base  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["shapley", "taylor", "apoz", "resnet-taylor", "resnet-apoz"])
    ap.add_argument("--layer", type=int, default=6)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--images", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if args.what.startswith("resnet"):
        from torchpruner_amd import get_resnet_pruning_graph
        from torchpruner_amd.models import resnet50
        model = resnet50().to(dev).eval()
        n = args.images or 8 * args.batch
        x = torch.randn(n, 3, 224, 224, device=dev)
        y = torch.randint(0, 1000, (n,), device=dev)
        mods = [m for m, _ in get_resnet_pruning_graph(model)]
    else:
        from torchpruner_amd.models import prunable_vgg16
        model = prunable_vgg16().to(dev).eval()
        n = args.images or (1000 if args.what == "shapley" else 200 * args.batch)
        x = torch.randn(n, 3, 32, 32, device=dev)
        y = torch.randint(0, 10, (n,), device=dev)
        mods = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    enq = {}
    orig = base.ScoreAccumulator.finalize

    def finalize(self, *a, **k):
        enq.setdefault("t", time.perf_counter())
        return orig(self, *a, **k)

    base.ScoreAccumulator.finalize = finalize
    # Shapley keeps its own fp64 column: its first host read (.cpu() / .item()) marks the end of enqueueing
    for name in ("cpu", "item"):
        fn = getattr(torch.Tensor, name)

        def wrapped(self, *a, _fn=fn, **k):
            if self.is_cuda:
                enq.setdefault("t", time.perf_counter())
            return _fn(self, *a, **k)

        setattr(torch.Tensor, name, wrapped)
    for rep in range(args.reps):
        enq.clear()
        dl = DeviceLoader(x, y, args.batch)
        if args.what == "shapley":
            m = ShapleyAttributionMetric(model, dl, F.cross_entropy, dev, sv_samples=5)
            run = lambda: m.run(mods[args.layer], find_best_evaluation_module=True)  # noqa: E731
        else:
            cls = APoZAttributionMetric if args.what.endswith("apoz") else TaylorAttributionMetric
            m = cls(model, dl, F.cross_entropy, dev)
            run = lambda: m.run_many(mods, find_best_evaluation_module=True)  # noqa: E731
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        host = enq.get("t", t0) - t0
        print(f"{args.what} rep {rep}: wall {wall * 1e3:.1f} ms, host until first finalize {host * 1e3:.1f} ms "
              f"(ratio {host / wall:.2f}); path {getattr(m, 'last_path', None)}", flush=True)


if __name__ == "__main__":
    main()
