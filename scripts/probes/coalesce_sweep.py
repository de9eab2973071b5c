"""B=100 VGG16 Taylor run_many (bench.py's vgg_taylor_b100_img_s setup: random-init weights,
synthetic batches) at several coalescing factors (TORCHPRUNER_COALESCE=k loader batches per engine
launch; 1 = the default element target). python scripts/probes/coalesce_sweep.py [--factors 1,10,20]"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--factors", default="1,10,20")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.models import prunable_vgg16
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(100 * args.steps, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (100 * args.steps,), device=dev)
    batches = [(x[i:i + 100], y[i:i + 100]) for i in range(0, x.shape[0], 100)]
    for f in args.factors.split(","):
        os.environ["TORCHPRUNER_COALESCE"] = f
        TaylorAttributionMetric(model, batches[:20], F.cross_entropy, dev).run_many(convs, True)  # tune
        for rep in range(2):
            m = TaylorAttributionMetric(model, batches, F.cross_entropy, dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.run_many(convs, True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"COALESCE={f} rep {rep}: {x.shape[0] / dt:.0f} img/s, {m.last_coalesce} batches/launch, "
                  f"path {m.last_path['path']}", flush=True)


if __name__ == "__main__":
    main()
