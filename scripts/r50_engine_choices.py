"""The ResNet-50 engine's kernel choices and step time at B=256 (bench.py config #3, random init,
synthetic batches): tunes on 2 batches, times --steps batches of APoZ (or --taylor), then prints
the tuner's choice per conv shape (cfg < 0: Winograd kinds of engine/fused_chain.py).
python scripts/r50_engine_choices.py [--steps 4] [--taylor]"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--taylor", action="store_true")
    args = ap.parse_args()
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import StreamLoader
    from torchpruner_amd.engine.fused_chain import TUNER
    from torchpruner_amd.models import resnet50
    dev = torch.device("cuda")
    torch.manual_seed(0)
    rn = resnet50().to(dev).eval().to(memory_format=torch.channels_last)
    mods = [m for m, _ in get_resnet_pruning_graph(rn)]
    M = TaylorAttributionMetric if args.taylor else APoZAttributionMetric
    M(rn, StreamLoader(2, 256, (3, 224, 224), 1000, dev, seed=1, channels_last=True), F.cross_entropy,
      dev).run_many(mods, find_best_evaluation_module=True)
    torch.cuda.synchronize()
    m = M(rn, StreamLoader(args.steps, 256, (3, 224, 224), 1000, dev, seed=2, channels_last=True),
          F.cross_entropy, dev)
    t0 = time.perf_counter()
    m.run_many(mods, find_best_evaluation_module=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{'taylor' if args.taylor else 'apoz'}: {dt / args.steps * 1e3:.2f} ms/step, "
          f"{256 * args.steps / dt:.0f} img/s, path {m.last_path['path']}", flush=True)
    for k, v in sorted(TUNER.cache.items(), key=lambda kv: str(kv[0])):
        print("  choice", k, "->", v)


if __name__ == "__main__":
    main()
