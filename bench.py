#!/usr/bin/env python
"""Headline benchmark: attribution images/sec (whole node), VGG16 Taylor; top-1 retained @ 50% pruned.

Workload (BASELINE.json config #2, scaled to N GPUs):
* VGG16-BN / CIFAR-10 shape (reference experiments/models/cifar10.py:62-77), random-init
  weights, eval mode, fp32 compute (the reference's precision).
* One step = Taylor attribution of one batch of B images *for every conv layer* (all 13
  units a 50%-filter prune needs), evaluated after BN+ReLU (``find_best_evaluation_module``),
  through the public API ``TaylorAttributionMetric.run_many``.
* Data parallel: one process per GPU (torchrun), whole batches sharded per rank, scores
  all-reduced over RCCL at the end of ``run_many`` (inside the timed region).
* Weak scaling: B images per GPU per step; ``value`` = total images/s over all GPUs.
* After timing (untimed): prune 50% of every conv layer's filters by the measured scores and
  report top-1 agreement with the unpruned model on held-out synthetic images
  (labels = the unpruned model's predictions, so top-1 before pruning is 100%).
* ``--baseline``: also time the reference-semantics eager implementation (one full pass per
  layer, clone + non-full backward hook, full backward, per-batch host numpy concat) on the
  same GPU for a few batches (rank 0), reported as ``eager_reference_img_s``.

Synthetic data of CIFAR-10 shape (no datasets in this environment).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from torchpruner_amd import Pruner, TaylorAttributionMetric, get_vgg_pruning_graph  # noqa: E402
from torchpruner_amd.data import DeviceLoader, teacher_labels  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.parallel import dist as pdist  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", 256)),
                    help="images per GPU per step")
    ap.add_argument("--baseline", action="store_true", help="also time the reference-semantics eager path")
    ap.add_argument("--baseline-batches", type=int, default=2)
    ap.add_argument("--no-prune", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args()


def log(*a):
    if pdist.get_rank() == 0:
        print(*a, file=sys.stderr, flush=True)


def make_batches(model, n_batches, B, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn(n_batches * B, 3, 32, 32, generator=g, device=device)
    y = teacher_labels(model, x, batch=1024)
    return x, y


def timed_run(metric, convs, world):
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores = metric.run_many(convs, find_best_evaluation_module=True)
    torch.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    return scores, dt


def main():
    args = parse()
    ctx = pdist.init_distributed()
    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    assert dev.type == "cuda", "bench.py needs a GPU"
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    B = args.batch

    # every rank builds the same global data set; each processes its own whole batches
    xw, yw = make_batches(model, max(args.warmup, 1) * world, B, dev, args.seed + 1)
    xt, yt = make_batches(model, args.steps * world, B, dev, args.seed + 2)
    warm = TaylorAttributionMetric(model, DeviceLoader(xw, yw, B), F.cross_entropy, dev)
    metric = TaylorAttributionMetric(model, DeviceLoader(xt, yt, B), F.cross_entropy, dev)

    _, _ = timed_run(warm, convs, world)  # warmup (untimed): W steps + the collective
    scores, dt = timed_run(metric, convs, world)
    total_imgs = args.steps * B * world
    value = total_imgs / dt
    ms_per_step = dt / args.steps * 1e3
    log(f"[bench] {world} GPU(s) x {args.steps} steps x B={B}: {dt*1e3:.1f} ms -> {value:.0f} img/s")

    result = {
        "metric": "attribution images/sec (whole node) VGG16 Taylor; top-1 retained @ 50% pruned",
        "value": round(value, 1),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (CIFAR-10 shape, random-init VGG16-BN, teacher labels)",
        "config": {
            "model": "VGG16-BN (CIFAR-10, reference classifier)",
            "global_batch": B * world,
            "per_gpu_batch": B,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "method": "TaylorAttributionMetric.run_many over 13 conv layers, find_best_evaluation_module=True",
        },
    }

    if args.baseline and rank == 0:
        from torchpruner_amd.bench.reference_semantics import reference_taylor_all
        nb = args.baseline_batches
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            ev = [find_best_module_for_attributions(model, c) for c in convs]
            dl = DeviceLoader(xt[: nb * B], yt[: nb * B], B)
            reference_taylor_all(model, DeviceLoader(xt[:B], yt[:B], B), F.cross_entropy, dev, ev[:1])  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reference_taylor_all(model, dl, F.cross_entropy, dev, ev)
            torch.cuda.synchronize()
            bt = time.perf_counter() - t0
        finally:
            os.environ.pop("TORCHPRUNER_BACKEND", None)
            model.zero_grad(set_to_none=True)
        result["eager_reference_img_s_per_gpu"] = round(nb * B / bt, 1)
        result["speedup_vs_eager_reference_per_gpu"] = round((value / world) / (nb * B / bt), 2)
        log(f"[bench] reference-semantics eager: {nb * B / bt:.0f} img/s per GPU")

    if not args.no_prune:
        # untimed: one-shot 50% filter pruning of every conv layer by the Taylor scores
        xv, yv = make_batches(model, 1, 1000, dev, args.seed + 3)
        conv_scores = {id(c): s for c, s in zip(convs, scores)}
        pruner = Pruner(model, (3, 32, 32), dev)
        for module, cascade in get_vgg_pruning_graph(model):
            if id(module) not in conv_scores:
                continue
            s = conv_scores[id(module)]
            idx = np.argsort(s, kind="stable")[: len(s) // 2]
            pruner.prune_model(module, idx, cascading_modules=cascade)
        with torch.no_grad():
            acc = (model(xv).argmax(1) == yv).float().mean().item()
        result["top1_retained_at_50pct"] = round(acc, 4)
        log(f"[bench] top-1 retained after 50% conv-filter pruning: {acc:.4f}")

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
