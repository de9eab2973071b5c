#!/usr/bin/env python
"""VGG16-BN / CIFAR-10 layerwise robustness study (reference notebook nbVGG:181-1584).

For each of the 15 prunable layers and each attribution method (WeightNorm, Random x3,
Sensitivity, Taylor, Taylor signed, APoZ, SV x3, SV mean+2std x3; nbVGG:251-263,1248) the
scores are computed with ``find_best_evaluation_module=True`` on 1,000 attribution images
(batch 100), units are removed in ascending-score order and loss/accuracy are measured on
1,000 test images after every removal; the AUC is the mean loss increase (nbVGG:1521-1527).

The reference run took 6 h 30 min on its GPU (nbVGG:1228-1229). Synthetic data: a briefly
trained VGG16-BN on the CIFAR-shaped prototype task (no CIFAR download in this environment),
so absolute AUCs differ from the paper's; the method ranking is what the study measures.

    python experiments/layerwise_robustness.py [--layers all|0,5,12] [--out results.json]
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchpruner_amd import (APoZAttributionMetric, RandomAttributionMetric,  # noqa: E402
                             SensitivityAttributionMetric, ShapleyAttributionMetric, TaylorAttributionMetric,
                             WeightNormAttributionMetric, get_vgg_pruning_graph)
from torchpruner_amd.data import DeviceLoader, PrototypeTask  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402
from torchpruner_amd.utils.ablation import ablation_auc, ablation_curve  # noqa: E402


def train(model, task, steps, seed=0):
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=0.05, total_steps=max(steps, 1))
    model.train()
    for i in range(steps):
        x, y = task.sample(128, seed * 7919 + i)
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(model(x), y).backward()
        opt.step()
        sched.step()
    model.eval()
    model.zero_grad(set_to_none=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="all")
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--sv-samples", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/layerwise_robustness.json")
    args = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(1)
    np.random.seed(1)
    model = prunable_vgg16().to(dev)
    task = PrototypeTask((3, 32, 32), 10, noise=2.0, seed=0, device=dev)
    train(model, task, args.train_steps)
    xa, ya = task.sample(1000, 101)
    xt, yt = task.sample(1000, 202)
    val_loader = DeviceLoader(xa, ya, 100)
    loss = F.cross_entropy
    methods = {
        "Weight Norm": WeightNormAttributionMetric(model, val_loader, loss, dev),
        "Random": RandomAttributionMetric(model, val_loader, loss, dev),
        "Sensitivity": SensitivityAttributionMetric(model, val_loader, loss, dev),
        "Taylor": TaylorAttributionMetric(model, val_loader, loss, dev),
        "Taylor signed": TaylorAttributionMetric(model, val_loader, loss, dev, signed=True),
        "APoZ": APoZAttributionMetric(model, val_loader, loss, dev),
        "SV": ShapleyAttributionMetric(model, val_loader, loss, dev, sv_samples=args.sv_samples),
        "SV mean+2std": ShapleyAttributionMetric(model, val_loader, loss, dev, sv_samples=args.sv_samples,
                                                 reduction=lambda x: np.mean(x, 0) + 2 * np.std(x, 0)),
    }
    graph = get_vgg_pruning_graph(model)
    layers = list(range(len(graph))) if args.layers == "all" else [int(v) for v in args.layers.split(",")]
    with torch.no_grad():
        base_loss = float(loss(model(xt), yt))
        base_acc = float((model(xt).argmax(1) == yt).float().mean())
    log = {"base_loss": base_loss, "base_acc": base_acc, "layers": {}}
    t_start = time.perf_counter()
    auc = {}
    for li in layers:
        module, _ = graph[len(graph) - 1 - li]  # graph is last-layer-first; li counts from the input
        name = next(n for n, m in model.named_modules() if m is module)
        ev = find_best_module_for_attributions(model, module)
        log["layers"][name] = {}
        for mname, metric in methods.items():
            runs = 3 if mname in ("Random", "SV", "SV mean+2std") else 1
            aucs = []
            t0 = time.perf_counter()
            for _ in range(runs):
                scores = metric.run(module, find_best_evaluation_module=True)
                ranking = np.argsort(scores, kind="stable")
                losses, accs = ablation_curve(model, ev, ranking, xt, yt, loss)
                aucs.append(ablation_auc(losses))
                n_units = len(ranking)
            dt = time.perf_counter() - t0
            log["layers"][name][mname] = {"auc": aucs, "seconds": round(dt, 3), "units": n_units,
                                         "acc_at_50pct": float(accs[n_units // 2])}
            a = auc.setdefault(mname, {"sum": np.zeros(runs), "count": 0})
            a["sum"] += np.array(aucs) * n_units
            a["count"] += n_units
            print(f"{name:14s} {mname:13s} AUC {np.mean(aucs):.4f} acc@50% {accs[n_units // 2]:.3f} "
                  f"({dt:.2f}s)", flush=True)
    total = time.perf_counter() - t_start
    log["auc"] = {m: {"mean": float(np.mean(v["sum"] / v["count"])), "std": float(np.std(v["sum"] / v["count"]))}
                  for m, v in auc.items()}
    log["wall_seconds"] = round(total, 2)
    log["reference_wall_seconds"] = 6 * 3600 + 30 * 60 + 2  # nbVGG:1228-1229 (all 15 layers)
    print(json.dumps(log["auc"], indent=1))
    print(f"total wall time {total:.1f}s for {len(layers)} layer(s)")
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(log, f, indent=1)


if __name__ == "__main__":
    main()
