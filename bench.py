#!/usr/bin/env python
"""Headline benchmark: attribution images/sec (whole node), VGG16 Taylor; top-1 retained @ 50% pruned.

Throughput (timed; BASELINE.json config #2, scaled to N GPUs):
* VGG16-BN / CIFAR-10 shape (reference experiments/models/cifar10.py:62-77), eval mode, fp32
  (the reference's precision), weights of a briefly trained teacher (untimed).
* One step = Taylor attribution of one batch of B images for EVERY conv layer (the 13 units a
  50%-filter prune needs), evaluated after BN+ReLU (``find_best_evaluation_module``), through the
  public API ``TaylorAttributionMetric.run_many``.
* Data parallel: one process per GPU (torchrun), whole batches sharded per rank (each rank
  materialises only its own batches), scores all-reduced over RCCL at the end of ``run_many``
  (inside the timed region). Weak scaling: B images per GPU per step; ``value`` = total img/s.
* ``vs_baseline``: the reference has no published number for this metric, so
  the comparison point is the reference algorithm run eagerly on the same GPU (one full pass
  per layer, activation clone + non-full backward hook, full backward, per-batch host numpy
  concatenation; ``bench/reference_semantics.py``), timed on rank 0 for a few batches.
  ``vs_baseline`` = per-GPU throughput / eager per-GPU throughput.

Accuracy (untimed; ``bench/prune_quality.py``, rank 0): the teacher is pruned for real —
``Pruner.prune_model`` through ``get_vgg_pruning_graph`` on every conv, 50% of the filters, in 4
increments per layer with a few SGD steps between increments (Molchanov-style iterative
pruning), Taylor scores vs Random scores under the same finetune budget.
``top1_retained_at_50pct`` = top-1 of the Taylor-pruned network / top-1 of the teacher, on held-out
samples, averaged over ``--quality-seeds`` seeds (each seed its own teacher and task draw). Training uses the deterministic native kernels with fixed configs, so the same seed
gives the same numbers in every run. ``top1_layerwise_mask_50pct_*``: the reference's
layerwise-robustness protocol at one point (nbVGG:1233-1285: each layer alone, lowest half of
its units zeroed after BN+ReLU; mean over layers).

Synthetic data of CIFAR-10 shape (no datasets in this environment).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.bench import prune_quality as pq  # noqa: E402
from torchpruner_amd.data import ShardLoader  # noqa: E402
from torchpruner_amd.parallel import dist as pdist  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402

METRIC = "attribution images/sec (whole node) VGG16 Taylor; top-1 retained @ 50% pruned"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", 2048)),
                    help="images per GPU per step (HBM-sized: small-spatial layers need >= 2k images to "
                         "fill 256 CUs)")
    ap.add_argument("--no-baseline", action="store_true", help="skip the reference-semantics eager timing")
    ap.add_argument("--baseline-batches", type=int, default=2)
    ap.add_argument("--no-prune", action="store_true", help="skip the (untimed) accuracy protocol")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--quality-seeds", type=int, default=3,
                    help="accuracy protocol over seeds seed..seed+K-1 (each its own teacher); top-1 figures "
                         "are means over the seeds, per-seed values are listed")
    ap.add_argument("--teacher-steps", type=int, default=pq.DEFAULTS["teacher_steps"])
    return ap.parse_args()


def log(*a):
    if pdist.get_rank() == 0:
        print(*a, file=sys.stderr, flush=True)


@torch.no_grad()
def layerwise_mask_top1(model, convs, scores, x, y, frac=0.5):
    """Reference layerwise-robustness protocol (nbVGG:1233-1285) at one point: for each conv
    layer alone, zero the ``frac`` lowest-scored channels after its BN+ReLU; mean top-1."""
    accs = []
    for conv, s in zip(convs, scores):
        idx = torch.as_tensor(np.argsort(s, kind="stable")[: int(len(s) * frac)], device=x.device)
        ev = find_best_module_for_attributions(model, conv)
        h = ev.register_forward_hook(lambda m, i, o, idx=idx: o.index_fill(1, idx, 0.0))
        try:
            accs.append(pq.top1(model, x, y))
        finally:
            h.remove()
    return float(np.mean(accs))


def timed_run(metric, convs, world):
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores = metric.run_many(convs, find_best_evaluation_module=True)
    torch.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = pdist.all_max_float(dt)
    return scores, dt


def main():
    args = parse()
    ctx = pdist.init_distributed()
    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    assert dev.type == "cuda", "bench.py needs a GPU"
    cfg = dict(pq.DEFAULTS, teacher_steps=args.teacher_steps)
    t0 = time.perf_counter()
    model, task = pq.make_teacher(args.seed, dev, cfg)  # deterministic: identical on every rank
    log(f"[bench] teacher: {cfg['teacher_steps']} SGD steps in {time.perf_counter() - t0:.1f}s (untimed)")
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    B = args.batch

    def loader(n_steps, seed):  # this rank's batches only (global batch i from seed i)
        return ShardLoader.build(lambda i: task.sample(B, seed * 1_000_003 + i), max(n_steps, 1) * world, B, rank,
                                 world)

    warm = TaylorAttributionMetric(model, loader(args.warmup, args.seed + 1), F.cross_entropy, dev)
    metric = TaylorAttributionMetric(model, loader(args.steps, args.seed + 2), F.cross_entropy, dev)
    _, _ = timed_run(warm, convs, world)  # warmup (untimed): W steps + the collective
    scores, dt = timed_run(metric, convs, world)
    assert metric.last_path["path"] == "fused", metric.last_path
    total_imgs = args.steps * B * world
    value = total_imgs / dt
    log(f"[bench] {world} GPU(s) x {args.steps} steps x B={B}: {dt * 1e3:.1f} ms -> {value:.0f} img/s "
        f"({metric.last_path['path']} path)")

    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic (CIFAR-10-shaped prototype-mixture task, {cfg['modes']} modes/class, noise "
                f"{cfg['noise']}; random-init VGG16-BN trained {cfg['teacher_steps']} steps, untimed)",
        "config": {
            "model": "VGG16-BN (CIFAR-10, reference classifier)",
            "global_batch": B * world,
            "per_gpu_batch": B,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "method": "TaylorAttributionMetric.run_many over 13 conv layers, find_best_evaluation_module=True",
        },
    }

    if not args.no_baseline and rank == 0:
        from torchpruner_amd.bench.reference_semantics import reference_taylor_all
        from torchpruner_amd.data import DeviceLoader
        nb = args.baseline_batches
        xb, yb = task.sample(nb * B, args.seed + 5)
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            ev = [find_best_module_for_attributions(model, c) for c in convs]
            reference_taylor_all(model, DeviceLoader(xb[:B], yb[:B], B), F.cross_entropy, dev, ev[:1])  # warm
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            reference_taylor_all(model, DeviceLoader(xb, yb, B), F.cross_entropy, dev, ev)
            torch.cuda.synchronize()
            bt = time.perf_counter() - t1
        finally:
            os.environ.pop("TORCHPRUNER_BACKEND", None)
            model.zero_grad(set_to_none=True)
        eager = nb * B / bt
        result["eager_reference_img_s_per_gpu"] = round(eager, 1)
        result["vs_baseline"] = round((value / world) / eager, 2)
        result["vs_baseline_definition"] = ("per-GPU img/s / reference-semantics eager img/s on the same GPU "
                                            "(BASELINE.md: the reference publishes no number for this metric)")
        log(f"[bench] reference-semantics eager: {eager:.0f} img/s per GPU -> vs_baseline {result['vs_baseline']}")

    if not args.no_prune and rank == 0:
        t1 = time.perf_counter()
        xv, yv = task.sample(cfg["val_imgs"], args.seed * 7 + 3)
        before = pq.top1(model, xv, yv)
        rng = np.random.RandomState(args.seed)
        lw_t = layerwise_mask_top1(model, convs, scores, xv, yv)
        lw_r = float(np.mean([layerwise_mask_top1(model, convs, [rng.random_sample(c.out_channels) for c in convs],
                                                  xv, yv) for _ in range(3)]))
        runs = [{"seed": args.seed, "top1_before": before}]
        for method in ("taylor", "random"):
            m = pq.iterative_prune(copy.deepcopy(model), task, method, args.seed, cfg)
            runs[0][f"top1_pruned_{method}"] = pq.top1(m, xv, yv)
            params = sum(p.numel() for p in m.parameters())
        for s in range(args.seed + 1, args.seed + max(1, args.quality_seeds)):
            runs.append(pq.run_protocol(s, dev, **cfg))  # its own teacher, task and held-out set
        mean = {k: float(np.mean([r[k] for r in runs])) for k in ("top1_before", "top1_pruned_taylor",
                                                                 "top1_pruned_random")}
        ret = {m: float(np.mean([r[f"top1_pruned_{m}"] / max(r["top1_before"], 1e-9) for r in runs]))
               for m in ("taylor", "random")}
        pruned = {m: mean[f"top1_pruned_{m}"] for m in ("taylor", "random")}
        before = mean["top1_before"]
        result.update({
            "top1_retained_at_50pct": round(ret["taylor"], 4),
            "top1_before": round(before, 4),
            "top1_pruned_50pct_taylor": round(pruned["taylor"], 4),
            "top1_pruned_50pct_random": round(pruned["random"], 4),
            "top1_retained_at_50pct_random": round(ret["random"], 4),
            "quality_seeds": [r["seed"] for r in runs],
            "top1_pruned_50pct_taylor_per_seed": [round(r["top1_pruned_taylor"], 4) for r in runs],
            "top1_pruned_50pct_random_per_seed": [round(r["top1_pruned_random"], 4) for r in runs],
            "params_before_after": [sum(p.numel() for p in model.parameters()), params],
            "prune_protocol": {k: cfg[k] for k in ("frac", "increments", "ft_steps", "final_ft_steps", "recal_batches",
                                                   "score_imgs", "val_imgs", "ft_lr", "noise")},
            "top1_layerwise_mask_50pct_taylor": round(lw_t, 4),
            "top1_layerwise_mask_50pct_random": round(lw_r, 4),
        })
        log(f"[bench] seeds {result['quality_seeds']}: mean top-1 before {before:.4f}; 50% of every conv pruned "
            f"(iterative, "
            f"{cfg['increments']} increments/layer, {cfg['ft_steps']} SGD steps each, +{cfg['final_ft_steps']}): "
            f"Taylor {pruned['taylor']:.4f}, Random {pruned['random']:.4f}; layerwise mask (nbVGG protocol): "
            f"Taylor {lw_t:.4f}, Random {lw_r:.4f} ({time.perf_counter() - t1:.1f}s untimed)")

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        pdist.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
