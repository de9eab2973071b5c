#!/usr/bin/env python
"""Config #5: ResNet-50 iterative prune -> finetune with DDP and optimizer-state rewiring.

Each round: (1) score every prunable bottleneck conv (conv1/conv2 of every block; the
residual-tied conv3/downsample are left intact, see get_resnet_pruning_graph) with a data-
parallel attribution metric (scores all-reduced over RCCL); (2) prune ``--frac`` of the
lowest-scored channels of each (indices broadcast from rank 0); (3) rebuild the DDP buckets
(PrunableDDP.rewrap) and finetune ``--steps`` SGD-momentum steps — the momentum buffers were
sliced together with the parameters by the pruner's multi-tensor gather.

    torchrun --nproc-per-node 8 experiments/prune_finetune.py --rounds 3 --frac 0.2
Synthetic data: a learnable prototype-mixture task (``PrototypeTask``, ``--classes`` classes at
``--res`` px) so the loss falls across rounds and held-out top-1 after every prune -> finetune
round is meaningful (random labels would leave the loss at ln(classes)); fp32.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--frac", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--score-batches", type=int, default=2)
    ap.add_argument("--metric", default="taylor", choices=["taylor", "apoz"])
    ap.add_argument("--res", type=int, default=112)
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--pretrain-steps", type=int, default=60, help="SGD steps before the first prune")
    ap.add_argument("--val-batches", type=int, default=4)
    ap.add_argument("--recal-batches", type=int, default=8,
                    help="BN running statistics re-estimated after each prune (same batches on every rank)")
    ap.add_argument("--convs", default="native", choices=["native", "library"],
                    help="native: training convolutions on the precompiled HIP kernels (engine/train.py); "
                         "library: MIOpen (JIT-compiles every new pruned shape)")
    args = ap.parse_args()
    ctx = pdist.init_distributed()
    dev, world = ctx.device, ctx.world_size
    torch.manual_seed(0)
    np.random.seed(0)
    model = resnet50(num_classes=args.classes).to(dev).to(memory_format=torch.channels_last)
    task = PrototypeTask((3, args.res, args.res), args.classes, noise=args.noise, seed=0, device=dev)
    val = task.stream(args.val_batches * world, args.batch, seed=999, channels_last=True)
    if args.convs == "native":
        from torchpruner_amd.engine.train import enable_native_convs
        enable_native_convs(model)
    wrapper = PrunableDDP(model, device=dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    pruner = Pruner(model, (3, args.res, args.res), dev, optimizer=opt)
    log = {"params": [count_parameters(model)], "rounds": []}
    t0 = time.perf_counter()
    pre_loss, _ = train(wrapper, dev, F.cross_entropy, task.stream(args.pretrain_steps * world, args.batch, seed=1,
                                                                   channels_last=True), opt, -1, log_every=0)
    _, pre_top1 = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
    if ctx.rank == 0:
        print(json.dumps({"pretrain_steps": args.pretrain_steps, "train_loss": round(pre_loss, 4),
                          "val_top1": round(pre_top1, 4), "s": round(time.perf_counter() - t0, 1)}), flush=True)
    for r in range(args.rounds):
        # (1) score every prunable conv data-parallel (scores all-reduced), (2) prune (indices
        # broadcast from rank 0; momentum buffers sliced with the parameters), (3) rebuild DDP
        # buckets, (4) re-estimate BN statistics on batches every rank shares, (5) finetune
        t1 = time.perf_counter()
        model.eval()
        sc_data = task.stream(args.score_batches * world, args.batch, seed=200 + r, channels_last=True)
        M = TaylorAttributionMetric if args.metric == "taylor" else APoZAttributionMetric
        graph = get_resnet_pruning_graph(model)
        scores = M(model, sc_data, F.cross_entropy, dev).run_many([m for m, _ in graph],
                                                                    find_best_evaluation_module=True)
        for (module, cascade), s in zip(graph, scores):
            k = int(len(s) * args.frac)
            if k > 0 and len(s) - k >= 8:
                pruner.prune_model(module, np.argsort(s, kind="stable")[:k], cascade)
        wrapper.rewrap()
        recalibrate_bn(model, task.stream(args.recal_batches, args.batch, seed=300 + r, channels_last=True))
        torch.cuda.synchronize()
        t_prune = time.perf_counter() - t1
        _, val_pruned = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        # warm-up steps absorb kernel selection for the new pruned shapes (MIOpen: JIT compilation)
        t0 = time.perf_counter()
        wu = task.stream(3 * world, args.batch, seed=50 + r, channels_last=True)
        train(wrapper, dev, F.cross_entropy, wu, opt, r, log_every=0)
        torch.cuda.synchronize()
        t_warm = time.perf_counter() - t0
        t0 = time.perf_counter()
        tr = task.stream(args.steps * world, args.batch, seed=100 + r, channels_last=True)
        loss, acc = train(wrapper, dev, F.cross_entropy, tr, opt, r, log_every=0)
        torch.cuda.synchronize()
        t_train = time.perf_counter() - t0
        _, val_ft = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        row = {"round": r, "params": count_parameters(model), "val_top1_after_prune": round(val_pruned, 4),
               "train_loss": round(loss, 4), "train_acc": round(acc, 4), "val_top1_after_finetune": round(val_ft, 4),
               "score_prune_recal_s": round(t_prune, 3), "warmup_compile_s": round(t_warm, 3),
               "train_s": round(t_train, 3), "train_img_s": round(args.steps * args.batch * world / t_train, 1),
               "in_sync": params_in_sync(model)}
        log["rounds"].append(row)
        if ctx.rank == 0:
            print(json.dumps(row), flush=True)
    if ctx.rank == 0:
        print(json.dumps({"params_start": log["params"][0], "params_end": count_parameters(model)}))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
