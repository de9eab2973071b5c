#!/usr/bin/env python
"""Headline benchmark: attribution images/sec (whole node), VGG16 Taylor; top-1 retained @ 50% pruned.

Workload (BASELINE.json config #2, scaled to N GPUs):
* VGG16-BN / CIFAR-10 shape (reference experiments/models/cifar10.py:62-77), random-init
  weights briefly trained (untimed, ``--train-steps``) on a synthetic CIFAR-shaped prototype
  task so that top-1 is meaningful; eval mode; fp32 compute (the reference's precision).
* One step = Taylor attribution of one batch of B images *for every conv layer* (all 13
  units a 50%-filter prune needs), evaluated after BN+ReLU (``find_best_evaluation_module``),
  through the public API ``TaylorAttributionMetric.run_many``.
* Data parallel: one process per GPU (torchrun), whole batches sharded per rank, scores
  all-reduced over RCCL at the end of ``run_many`` (inside the timed region).
* Weak scaling: B images per GPU per step; ``value`` = total images/s over all GPUs.
* After timing (untimed): prune 50% of every conv layer's filters by the measured scores
  (one shot, no finetuning) and report held-out top-1 before/after, plus the same prune with
  Random scores as a reference point.
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
from torchpruner_amd.data import DeviceLoader, PrototypeTask  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.parallel import dist as pdist  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", 2048)),
                    help="images per GPU per step (HBM-sized: small-spatial layers need >= 2k images to "
                         "fill 256 CUs; 512 -> 148k, 1024 -> 156k, 2048 -> 162k img/s on one MI355X)")
    ap.add_argument("--baseline", action="store_true", help="also time the reference-semantics eager path")
    ap.add_argument("--baseline-batches", type=int, default=2)
    ap.add_argument("--no-prune", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--train-steps", type=int, default=int(os.environ.get("BENCH_TRAIN_STEPS", 300)),
                    help="untimed SGD steps on the synthetic task before scoring (0 = random init)")
    ap.add_argument("--finetune-steps", type=int, default=int(os.environ.get("BENCH_FINETUNE_STEPS", 100)),
                    help="untimed SGD steps after the one-shot all-layer 50%% prune (Taylor and Random alike)")
    ap.add_argument("--task-noise", type=float, default=2.0, help="per-pixel noise of the synthetic prototype task")
    ap.add_argument("--task-modes", type=int, default=8,
                    help="prototypes per class: a mixture task that needs VGG16's capacity, so pruning half of "
                         "a layer costs accuracy and scoring methods separate (profiles/taylor_quality_sweep.txt)")
    return ap.parse_args()


def log(*a):
    if pdist.get_rank() == 0:
        print(*a, file=sys.stderr, flush=True)


def train_teacher(model, task, steps, device, seed):
    """Untimed: a few hundred SGD steps (reference optimizer settings, cifar10.py:95-99) on the
    synthetic prototype task; all ranks end with rank 0's weights."""
    if steps > 0:
        opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=0.05, total_steps=steps)
        model.train()
        for i in range(steps):
            x, y = task.sample(128, seed * 100_003 + i)
            opt.zero_grad(set_to_none=True)
            F.cross_entropy(model(x), y).backward()
            opt.step()
            sched.step()
    model.eval()
    model.zero_grad(set_to_none=True)
    if pdist.get_world_size() > 1:
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                pdist.broadcast_tensor_(t.data, 0)


@torch.no_grad()
def layerwise_top1(model, convs, scores, x, y, frac=0.5):
    """Reference layerwise-robustness protocol (nbVGG:1233-1285) at one point: for each conv
    layer alone, zero the ``frac`` lowest-scored channels after its BN+ReLU; mean top-1."""
    from torchpruner_amd.utils import find_best_module_for_attributions
    accs = []
    for conv, s in zip(convs, scores):
        idx = torch.as_tensor(np.argsort(s, kind="stable")[: int(len(s) * frac)], device=x.device)
        ev = find_best_module_for_attributions(model, conv)
        h = ev.register_forward_hook(lambda m, i, o, idx=idx: o.index_fill(1, idx, 0.0))
        try:
            accs.append(top1(model, x, y))
        finally:
            h.remove()
    return float(np.mean(accs))


@torch.no_grad()
def top1(model, x, y):
    model.eval()
    return float((model(x).argmax(1) == y).float().mean())


def prune_half(model, scores_by_conv, dev):
    pruner = Pruner(model, (3, 32, 32), dev)
    for module, cascade in get_vgg_pruning_graph(model):
        s = scores_by_conv.get(id(module))
        if s is None:
            continue
        idx = np.argsort(s, kind="stable")[: len(s) // 2]
        pruner.prune_model(module, idx, cascading_modules=cascade)


def finetune(model, task, steps, seed):
    """Untimed: a short SGD finetune of a pruned model (the reference's train loop shape,
    experiments/utils/train.py:11-48) on the native training convolutions, so the new pruned
    shapes need no MIOpen JIT. Taylor- and Random-pruned models see the same batches."""
    from torchpruner_amd.engine.train import native_convs
    if steps <= 0:
        return
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    model.train()
    with native_convs(model):
        for i in range(steps):
            x, y = task.sample(128, seed * 100_003 + 77_777 + i)
            opt.zero_grad(set_to_none=True)
            F.cross_entropy(model(x), y).backward()
            opt.step()
    model.eval()
    model.zero_grad(set_to_none=True)


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
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    model = prunable_vgg16().to(dev)
    task = PrototypeTask((3, 32, 32), 10, noise=args.task_noise, seed=args.seed, device=dev,
                         modes_per_class=args.task_modes)
    t0 = time.perf_counter()
    train_teacher(model, task, args.train_steps, dev, args.seed)
    log(f"[bench] teacher: {args.train_steps} SGD steps in {time.perf_counter() - t0:.1f}s (untimed)")
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    B = args.batch

    # every rank builds the same global data set; each processes its own whole batches
    xw, yw = task.sample(max(args.warmup, 1) * world * B, args.seed + 1)
    xt, yt = task.sample(args.steps * world * B, args.seed + 2)
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
        "data": "synthetic (CIFAR-10-shaped prototype-mixture task, 8 modes/class; random-init VGG16-BN "
                "briefly trained, untimed)",
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
        # untimed: one-shot 50% filter pruning of every conv layer (no finetuning)
        import copy
        xv, yv = task.sample(2000, args.seed + 3)
        before = top1(model, xv, yv)
        rng = np.random.RandomState(args.seed)
        lw_taylor = layerwise_top1(model, convs, scores, xv, yv)
        lw_random = float(np.mean([layerwise_top1(model, convs, [rng.random_sample(c.out_channels) for c in convs],
                                                  xv, yv) for _ in range(3)]))
        result["top1_layerwise_50pct_taylor"] = round(lw_taylor, 4)
        result["top1_layerwise_50pct_random"] = round(lw_random, 4)
        log(f"[bench] layerwise 50% (one layer at a time, mean over 13): Taylor {lw_taylor:.4f}, "
            f"Random {lw_random:.4f} (mean of 3 draws)")
        rnd = copy.deepcopy(model)
        prune_half(model, {id(c): s for c, s in zip(convs, scores)}, dev)
        after = top1(model, xv, yv)
        rconvs = [m for m in rnd.features if isinstance(m, torch.nn.Conv2d)]
        rng = np.random.RandomState(args.seed)
        prune_half(rnd, {id(c): rng.random_sample(c.out_channels) for c in rconvs}, dev)
        after_rnd = top1(rnd, xv, yv)
        result["top1_before"] = round(before, 4)
        result["top1_oneshot_all_layers_50pct_taylor"] = round(after, 4)
        result["top1_retained_at_50pct"] = round(lw_taylor / max(before, 1e-9), 4)
        result["top1_oneshot_all_layers_50pct_random"] = round(after_rnd, 4)
        log(f"[bench] top-1 before {before:.4f}; after one-shot 50% prune of ALL conv layers (no finetune): "
            f"Taylor {after:.4f}, Random {after_rnd:.4f}")
        if args.finetune_steps > 0:
            finetune(model, task, args.finetune_steps, args.seed)
            finetune(rnd, task, args.finetune_steps, args.seed)
            ft, ft_rnd = top1(model, xv, yv), top1(rnd, xv, yv)
            result["finetune_steps"] = args.finetune_steps
            result["top1_oneshot_50pct_finetuned_taylor"] = round(ft, 4)
            result["top1_oneshot_50pct_finetuned_random"] = round(ft_rnd, 4)
            log(f"[bench] after {args.finetune_steps} finetune SGD steps (B=128, untimed): "
                f"Taylor {ft:.4f}, Random {ft_rnd:.4f}")

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
