#!/usr/bin/env python
"""Config #5: ResNet-50 iterative prune -> finetune with DDP and optimizer-state rewiring, and a
method comparison at equal budgets (the point of the reference's studies: nbVGG:1233-1285,
AUC table nbVGG:1560-1575; iterative loop nbUNT:169-193; momentum rewire test_pruner.py:205-228).

Each round: (1) score every prunable bottleneck conv (conv1/conv2 of every block; the
residual-tied conv3/downsample are left intact, see get_resnet_pruning_graph) with a data-
parallel attribution metric (scores all-reduced over RCCL; ``random`` draws uniform scores on
rank 0); (2) prune ``--frac`` of the lowest-scored channels of each (indices broadcast from rank
0); (3) rebuild the DDP buckets (PrunableDDP.rewrap), re-estimate BN statistics, and finetune
``--steps`` SGD-momentum steps — the momentum buffers were sliced together with the parameters by
the pruner's multi-tensor gather.

    torchrun --nproc-per-node 8 experiments/prune_finetune.py --rounds 3 --frac 0.2
    python experiments/prune_finetune.py --compare taylor,apoz,random --seeds 0,1,2 --classes 20 --modes 8 \
        --noise 2.5 --teacher-target 0.85 --pretrain-steps 400 --rounds 3 --steps 15

``--compare``: for every seed one teacher is trained (``--pretrain-steps``), then EVERY method
prunes a copy of that same teacher with the same budgets (rounds, fraction, finetune steps,
batches); the JSON lines report val top-1 after each prune and after each finetune, and a final
summary line gives per-method means and standard deviations over seeds.

Synthetic data: a learnable prototype-mixture task (``PrototypeTask``: ``--classes`` classes of
``--modes`` prototypes each at ``--res`` px, additive noise ``--noise``) sized so the unpruned
network is accurate but not saturated; fp32.
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

from torchpruner_amd import APoZAttributionMetric, Pruner, TaylorAttributionMetric, get_resnet_pruning_graph  # noqa
from torchpruner_amd.data import PrototypeTask  # noqa: E402
from torchpruner_amd.models import resnet50  # noqa: E402
from torchpruner_amd.parallel import PrunableDDP, dist as pdist, params_in_sync  # noqa: E402
from torchpruner_amd.utils import count_parameters, recalibrate_bn, test, train  # noqa: E402

METRICS = {"taylor": TaylorAttributionMetric, "apoz": APoZAttributionMetric, "random": None}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--frac", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--score-batches", type=int, default=2)
    ap.add_argument("--metric", default="taylor", choices=sorted(METRICS))
    ap.add_argument("--compare", default=None, help="comma-separated methods pruned from the same teacher, e.g. "
                                                     "taylor,apoz,random")
    ap.add_argument("--seeds", default="0", help="comma-separated seeds (teacher init, task draw, batches)")
    ap.add_argument("--res", type=int, default=112)
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--modes", type=int, default=1, help="prototypes per class (task difficulty)")
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--pretrain-steps", type=int, default=60, help="SGD steps before the first prune (max with "
                                                                   "--teacher-target)")
    ap.add_argument("--teacher-target", type=float, default=None,
                    help="stop pretraining once val top-1 reaches this (checked every --check-every steps): an "
                         "unsaturated teacher, so recovery and method differences stay measurable")
    ap.add_argument("--check-every", type=int, default=20)
    ap.add_argument("--val-batches", type=int, default=4)
    ap.add_argument("--recal-batches", type=int, default=8,
                    help="BN running statistics re-estimated after each prune (same batches on every rank)")
    ap.add_argument("--convs", default="native", choices=["native", "library"],
                    help="native: training convolutions on the precompiled HIP kernels (engine/train.py); "
                         "library: MIOpen (JIT-compiles every new pruned shape)")
    return ap.parse_args()


def build(args, dev, seed, state=None):
    """ResNet-50 (channels_last, native training convs), its DDP wrapper, SGD and the pruner."""
    torch.manual_seed(seed)
    model = resnet50(num_classes=args.classes).to(dev).to(memory_format=torch.channels_last)
    if state is not None:
        model.load_state_dict(state)
    if args.convs == "native":
        from torchpruner_amd.engine.train import enable_native_convs
        enable_native_convs(model)
    wrapper = PrunableDDP(model, device=dev)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-4)
    pruner = Pruner(model, (3, args.res, args.res), dev, optimizer=opt)
    return model, wrapper, opt, pruner


def prune_rounds(args, model, wrapper, opt, pruner, task, val, method, seed, world, rank, emit):
    """The iterative prune -> finetune loop; returns the per-round rows."""
    dev = next(model.parameters()).device
    rng = np.random.RandomState(seed * 7919 + 17)
    rows = []
    for r in range(args.rounds):
        # (1) score every prunable conv data-parallel (scores all-reduced), (2) prune (indices
        # broadcast from rank 0; momentum buffers sliced with the parameters), (3) rebuild DDP
        # buckets, (4) re-estimate BN statistics on batches every rank shares, (5) finetune
        t1 = time.perf_counter()
        model.eval()
        graph = get_resnet_pruning_graph(model)
        if METRICS[method] is None:
            scores = [rng.random_sample(m.out_channels) for m, _ in graph]
        else:
            sc_data = task.stream(args.score_batches * world, args.batch, seed=seed * 1000 + 200 + r,
                                  channels_last=True)
            scores = METRICS[method](model, sc_data, F.cross_entropy, dev).run_many(
                [m for m, _ in graph], find_best_evaluation_module=True)
        for (module, cascade), s in zip(graph, scores):
            k = int(len(s) * args.frac)
            if k > 0 and len(s) - k >= 8:
                pruner.prune_model(module, np.argsort(s, kind="stable")[:k], cascade)
        wrapper.rewrap()
        recalibrate_bn(model, task.stream(args.recal_batches, args.batch, seed=seed * 1000 + 300 + r,
                                          channels_last=True))
        torch.cuda.synchronize()
        t_prune = time.perf_counter() - t1
        _, val_pruned = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        # warm-up steps absorb kernel selection for the new pruned shapes (MIOpen: JIT compilation)
        t0 = time.perf_counter()
        wu = task.stream(3 * world, args.batch, seed=seed * 1000 + 50 + r, channels_last=True)
        train(wrapper, dev, F.cross_entropy, wu, opt, r, log_every=0)
        torch.cuda.synchronize()
        t_warm = time.perf_counter() - t0
        t0 = time.perf_counter()
        tr = task.stream(args.steps * world, args.batch, seed=seed * 1000 + 100 + r, channels_last=True)
        loss, acc = train(wrapper, dev, F.cross_entropy, tr, opt, r, log_every=0)
        torch.cuda.synchronize()
        t_train = time.perf_counter() - t0
        _, val_ft = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        row = {"method": method, "seed": seed, "round": r, "params": count_parameters(model),
               "val_top1_after_prune": round(val_pruned, 4), "train_loss": round(loss, 4),
               "val_top1_after_finetune": round(val_ft, 4), "score_prune_recal_s": round(t_prune, 3),
               "warmup_compile_s": round(t_warm, 3), "train_s": round(t_train, 3),
               "train_img_s": round(args.steps * args.batch * world / t_train, 1), "in_sync": params_in_sync(model)}
        rows.append(row)
        emit(row)
    return rows


def main():
    args = parse()
    ctx = pdist.init_distributed()
    dev, world, rank = ctx.device, ctx.world_size, ctx.rank

    def emit(obj):
        if rank == 0:
            print(json.dumps(obj), flush=True)

    methods = args.compare.split(",") if args.compare else [args.metric]
    for m in methods:
        assert m in METRICS, f"unknown method {m}"
    seeds = [int(s) for s in args.seeds.split(",")]
    all_rows, teachers = [], []
    for seed in seeds:
        np.random.seed(seed)
        task = PrototypeTask((3, args.res, args.res), args.classes, noise=args.noise, seed=seed, device=dev,
                             modes_per_class=args.modes)
        val = task.stream(args.val_batches * world, args.batch, seed=seed * 1000 + 999, channels_last=True)
        model, wrapper, opt, pruner = build(args, dev, seed)
        t0 = time.perf_counter()
        done, part = 0, 0
        while done < args.pretrain_steps:
            n = args.pretrain_steps - done if args.teacher_target is None else min(args.check_every,
                                                                                   args.pretrain_steps - done)
            pre_loss, _ = train(wrapper, dev, F.cross_entropy, task.stream(n * world, args.batch,
                                                                           seed=seed * 1000 + 1 + 7 * part,
                                                                           channels_last=True), opt, -1, log_every=0)
            done += n
            part += 1
            _, pre_top1 = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
            if args.teacher_target is not None and pre_top1 >= args.teacher_target:
                break
        emit({"seed": seed, "pretrain_steps": done, "train_loss": round(pre_loss, 4),
              "val_top1": round(pre_top1, 4), "params": count_parameters(model), "s": round(time.perf_counter() - t0, 1)})
        teachers.append(round(pre_top1, 4))
        if len(methods) == 1:
            all_rows += prune_rounds(args, model, wrapper, opt, pruner, task, val, methods[0], seed, world, rank, emit)
            continue
        from torchpruner_amd.engine.train import disable_native_convs
        disable_native_convs([mm for mm in model.modules() if "forward" in mm.__dict__])
        teacher = {k: v.detach().clone() for k, v in model.state_dict().items()}
        del model, wrapper, opt, pruner
        for method in methods:
            m2, w2, o2, p2 = build(args, dev, seed, teacher)
            rows = prune_rounds(args, m2, w2, o2, p2, task, val, method, seed, world, rank, emit)
            for row in rows:
                row["teacher_val_top1"] = round(pre_top1, 4)
            all_rows += rows
            del m2, w2, o2, p2
    if len(methods) > 1:
        summary = {}
        for method in methods:
            per_round = []
            for r in range(args.rounds):
                pr = [x["val_top1_after_prune"] for x in all_rows if x["method"] == method and x["round"] == r]
                ft = [x["val_top1_after_finetune"] for x in all_rows if x["method"] == method and x["round"] == r]
                per_round.append({"round": r, "after_prune_mean": round(float(np.mean(pr)), 4),
                                  "after_prune_std": round(float(np.std(pr)), 4),
                                  "after_finetune_mean": round(float(np.mean(ft)), 4),
                                  "after_finetune_std": round(float(np.std(ft)), 4)})
            summary[method] = per_round
        # separation of each method from random in units of the seeds' spread (per round, after prune)
        sep = {}
        if "random" in methods:
            for method in methods:
                if method == "random":
                    continue
                sep[method] = []
                for r in range(args.rounds):
                    a = [x["val_top1_after_prune"] for x in all_rows if x["method"] == method and x["round"] == r]
                    b = [x["val_top1_after_prune"] for x in all_rows if x["method"] == "random" and x["round"] == r]
                    spread = float(np.sqrt(np.var(a) + np.var(b))) or 1e-9
                    sep[method].append(round((float(np.mean(a)) - float(np.mean(b))) / spread, 2))
        emit({"summary": summary, "teacher_top1": teachers, "separation_vs_random_after_prune": sep, "seeds": seeds,
              "rounds": args.rounds, "frac": args.frac, "steps": args.steps, "world": world,
              "task": {"classes": args.classes, "modes": args.modes, "noise": args.noise, "res": args.res}})
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
