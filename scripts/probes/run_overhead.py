"""Per-run fixed cost of TaylorAttributionMetric.run_many on the fused VGG engine: times runs of
1, 5 and 20 batches (B images each), fits t = a + b * n, and profiles the host side of one
1-batch run (cProfile, top functions by cumulative time).
Usage: python scripts/probes/run_overhead.py [--batch 2048]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    B = args.batch
    x = torch.randn(20 * B, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (20 * B,), device=dev)

    def run(n):
        m = TaylorAttributionMetric(model, DeviceLoader(x[:n * B], y[:n * B], B), F.cross_entropy, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.run_many(convs, find_best_evaluation_module=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for n in (1, 5, 20):
        run(n)  # warm (autotune, graphs of nothing, allocator)
    res = {n: min(run(n) for _ in range(3)) for n in (1, 5, 20)}
    b = (res[20] - res[5]) / 15
    a = res[20] - 20 * b
    print(f"B={B}: " + " ".join(f"{n} batches {t * 1e3:.2f} ms" for n, t in res.items())
          + f" -> per batch {b * 1e3:.3f} ms, per run {a * 1e3:.2f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    run(1)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
