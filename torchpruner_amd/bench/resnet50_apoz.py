"""Config #3: ResNet-50 / ImageNet-shape synthetic, APoZAttributionMetric, data parallel with the
per-unit scores all-reduced over RCCL (one collective per run).

    python -m torchpruner_amd.bench.resnet50_apoz [--batch 256] [--steps 10]
    torchrun --nproc-per-node 8 -m torchpruner_amd.bench.resnet50_apoz ...

One pass scores every prunable conv of every bottleneck (``run_many``): the whole network runs
on the ResNet engine (engine/resnet_engine.py: implicit-GEMM / Winograd MFMA convs with the
eval-mode BN folded in, residual + ReLU fused in the epilogues) and the APoZ counts of every
evaluation BN come out of the conv epilogues; ``--metric taylor|sensitivity`` adds the engine's
input-gradient-only backward. ``metric.last_path`` is asserted to be the engine. fp32; synthetic
data (batch i regenerated on device from a seed).
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.nn.functional as F

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, TaylorAttributionMetric,
                             get_resnet_pruning_graph)
from torchpruner_amd.data import StreamLoader
from torchpruner_amd.models import resnet50
from torchpruner_amd.parallel import dist as pdist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--metric", default="apoz", choices=["apoz", "taylor", "sensitivity"])
    args = ap.parse_args()
    M = {"apoz": APoZAttributionMetric, "taylor": TaylorAttributionMetric,
         "sensitivity": SensitivityAttributionMetric}[args.metric]
    ctx = pdist.init_distributed()
    dev, world = ctx.device, ctx.world_size
    torch.manual_seed(0)
    model = resnet50().to(dev).eval()
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    modules = [m for m, _ in get_resnet_pruning_graph(model)]
    warm = StreamLoader(args.warmup * world, args.batch, (3, 224, 224), 1000, dev, seed=1,
                        channels_last=bool(args.channels_last))
    data = StreamLoader(args.steps * world, args.batch, (3, 224, 224), 1000, dev, seed=2,
                        channels_last=bool(args.channels_last))
    M(model, warm, F.cross_entropy, dev).run_many(modules, find_best_evaluation_module=True)
    metric = M(model, data, F.cross_entropy, dev)
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores = metric.run_many(modules, find_best_evaluation_module=True)
    torch.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    assert metric.last_path["path"] == "resnet", metric.last_path
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    if ctx.rank == 0:
        print(json.dumps({"metric": f"{M.__name__} attribution images/sec (whole node), ResNet-50 224x224",
                          "value": round(args.steps * args.batch * world / dt, 1), "unit": "images/s",
                          "n_gpus": world, "per_gpu_batch": args.batch, "steps": args.steps,
                          "path": metric.last_path["path"],
                          "modules_scored": len(modules), "dtype": "fp32", "data": "synthetic",
                          "units_total": int(sum(len(s) for s in scores))}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
