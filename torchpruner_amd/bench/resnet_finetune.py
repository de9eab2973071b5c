"""BASELINE config #5 inside ``bench.py``: ResNet-50 iterative prune -> finetune under DDP.

Two measurements, every rank taking part (one process per GPU, RCCL):

``finetune_throughput`` — the training step the loop spends its time in, AFTER a prune:
ResNet-50 (ImageNet shape, 224 px, random init synced from rank 0) on the native training
kernels (engine/train.py) inside :class:`PrunableDDP`, SGD with momentum. A few steps create the
momentum buffers; then every prunable bottleneck conv (get_resnet_pruning_graph) loses ``frac``
of its filters by data-parallel Taylor scores (indices broadcast from rank 0, R5; parameters,
gradients and momentum sliced by the pruner's multi-tensor gather), the DDP buckets are rebuilt
(``rewrap``, R7), the new shapes warm up, and ``steps`` DDP steps (forward, backward, bucketed
gradient all-reduce over RCCL (R6), optimizer step) are timed between barriers. Weak scaling:
``batch`` images per GPU per step; the value is whole-node images/s. Reference loop:
nbUNT:169-193, experiments/utils/train.py:11-48, momentum rewire test_pruner.py:205-228.

``prune_finetune_quality`` — one prune -> finetune round, Taylor vs Random from the SAME teacher:
a 20-class prototype-mixture task at 112 px sized so the teacher is accurate but not saturated;
the teacher trains identically on every rank (native deterministic kernels, fixed kernel
choices) and is then synced; each method prunes ``frac`` of every prunable conv of a copy,
re-estimates BN statistics on batches every rank shares, and finetunes under DDP; val top-1 is
reported after the prune and after the finetune (all-reduced over ranks, R8).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F

from .. import Pruner, TaylorAttributionMetric, get_resnet_pruning_graph
from ..data import PrototypeTask, StreamLoader
from ..engine.fused_chain import TUNER
from ..engine.train import disable_native_convs, enable_native_convs
from ..models import resnet50
from ..parallel import PrunableDDP, params_in_sync
from ..parallel import dist as pdist
from ..utils import count_parameters, recalibrate_bn, test, train


def _prune_all(model, pruner, scores, frac):
    """Prune ``frac`` of the lowest-scored filters of every prunable conv (indices synced, R5)."""
    for (module, cascade), s in zip(get_resnet_pruning_graph(model), scores):
        k = int(len(s) * frac)
        if k > 0 and len(s) - k >= 8:
            pruner.prune_model(module, np.argsort(s, kind="stable")[:k], cascade)


def _timed(fn, world):
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    return out, (pdist.all_max_float(dt) if world > 1 else dt)


def _sgd(params, lr, dev):
    """SGD momentum 0.9, wd 1e-4 (the finetune recipe); torch's fused kernel on the GPU (one
    launch per step instead of ~13 multi-tensor foreach launches, +1.5% on the ResNet-50 step)."""
    params = list(params)
    kw = {"fused": True} if torch.device(dev).type == "cuda" else {}
    return torch.optim.SGD(params, lr=lr, momentum=0.9, weight_decay=1e-4, **kw)


def finetune_throughput(dev, world, rank, steps=10, warmup=3, batch=128, res=224, frac=0.2, seed=0,
                        score_batch=64, rounds=2):
    torch.manual_seed(seed)
    model = resnet50().to(dev).to(memory_format=torch.channels_last)
    sync = pdist.sync_module(model)
    enable_native_convs(model)
    wrapper = PrunableDDP(model, device=dev)
    opt = _sgd(model.parameters(), 0.01, dev)
    pruner = Pruner(model, (3, res, res), dev, optimizer=opt)
    shape = (3, res, res)

    def stream(n, s, bs=batch):
        return StreamLoader(n * world, bs, shape, 1000, dev, seed=s, channels_last=True)

    params0 = count_parameters(model)
    train(wrapper, dev, F.cross_entropy, stream(2, seed + 1), opt, 0, log_every=0)  # momentum buffers exist
    _, dt_dense = _timed(lambda: train(wrapper, dev, F.cross_entropy, stream(steps, seed + 2), opt, 0, log_every=0),
                         world)
    # the iterative loop (nbUNT:169-193 prunes layer after layer, then trains): ``rounds`` rounds
    # of [data-parallel Taylor scores -> prune frac of every prunable conv (parameters, grads and
    # momentum sliced, R5) -> DDP rewrap (R7) -> new-shape warm-up -> timed finetune segment]
    per_round, t_prune, t_warm, tot_imgs, tot_dt, loss = [], [], [], 0, 0.0, float("nan")
    for r in range(rounds):
        t0 = time.perf_counter()
        model.eval()
        graph = get_resnet_pruning_graph(model)
        scores = TaylorAttributionMetric(model, stream(1, seed + 3 + 10 * r, score_batch), F.cross_entropy,
                                         dev).run_many([m for m, _ in graph], find_best_evaluation_module=True)
        _prune_all(model, pruner, scores, frac)
        wrapper.rewrap()
        t_prune.append(round(time.perf_counter() - t0, 2))
        t0 = time.perf_counter()
        train(wrapper, dev, F.cross_entropy, stream(warmup, seed + 4 + 10 * r), opt, 1, log_every=0)  # new shapes
        torch.cuda.synchronize()
        t_warm.append(round(time.perf_counter() - t0, 2))
        (loss, _), dt = _timed(lambda: train(wrapper, dev, F.cross_entropy, stream(steps, seed + 5 + 10 * r), opt,
                                             1, log_every=0), world)
        per_round.append({"round": r + 1, "img_s": round(steps * batch * world / dt, 1),
                          "params": count_parameters(model), "in_sync": params_in_sync(model)})
        tot_imgs += steps * batch * world
        tot_dt += dt
    dt = tot_dt / rounds
    out = {
        "resnet50_finetune_img_s": round(tot_imgs / tot_dt, 1),
        "resnet50_train_dense_img_s": round(steps * batch * world / dt_dense, 1),
        "resnet50_finetune_config": {
            "per_gpu_batch": batch, "image": list(shape), "steps": steps, "warmup": warmup, "dtype": "fp32",
            "prune": f"{rounds} rounds, each {frac:.0%} of every prunable bottleneck conv (conv1/conv2) by Taylor "
                     "scores, then DDP rewrap and a timed finetune segment; the value is over all rounds",
            "rounds": per_round,
            "params_before_after": [params0, count_parameters(model)], "optimizer": "SGD momentum 0.9, wd 1e-4 (torch fused kernel on GPU)",
            "ddp": f"PrunableDDP (bucket_cap_mb={wrapper.bucket_cap_mb}), rewrapped after every prune",
            "kernels": "native training convs / BN (engine/train.py)", "prune_rewrap_s": t_prune,
            "new_shape_warmup_s": t_warm, "in_sync": params_in_sync(model),
            "weights_agreed_before_broadcast": sync["agreed_before"], "loss_finite": bool(np.isfinite(loss))},
    }
    disable_native_convs([m for m in model.modules() if "forward" in m.__dict__])
    return out


# teacher: early stop at val top-1 >= 0.85 (checked every 25 steps); 8% label noise caps it at ~0.92
# (as bench/prune_quality.py), so it cannot saturate at 1.0 even when the task is learnt quickly
QUALITY = dict(res=112, classes=20, modes=8, noise=2.5, label_noise=0.08, batch=64, teacher_target=0.85,
               teacher_max_steps=800, check_every=25, frac=0.2, ft_steps=60, recal_batches=8, val_batches=8,
               score_batches=4, lr=0.01, ft_lr=0.002)


def prune_finetune_quality(dev, world, rank, seed=0, cfg=None):
    cfg = dict(QUALITY, **(cfg or {}))
    shape = (3, cfg["res"], cfg["res"])
    task = PrototypeTask(shape, cfg["classes"], noise=cfg["noise"], seed=seed, device=dev,
                         modes_per_class=cfg["modes"], label_noise=cfg["label_noise"])
    val = task.stream(cfg["val_batches"] * world, cfg["batch"], seed=seed * 1000 + 999, channels_last=True)
    t0 = time.perf_counter()
    with TUNER.fixed():  # deterministic kernel choices: every rank trains the same teacher
        torch.manual_seed(seed)
        teacher = resnet50(num_classes=cfg["classes"]).to(dev).to(memory_format=torch.channels_last)
        enable_native_convs(teacher)
        opt = _sgd(teacher.parameters(), cfg["lr"], dev)
        done, part, top1 = 0, 0, 0.0
        while done < cfg["teacher_max_steps"] and top1 < cfg["teacher_target"]:
            n = min(cfg["check_every"], cfg["teacher_max_steps"] - done)
            # the same batches on every rank, no DDP: identical replicas without communication
            train(teacher, dev, F.cross_entropy, task.stream(n, cfg["batch"], seed=seed * 1000 + 1 + 7 * part,
                                                              channels_last=True), opt, -1, log_every=0, shard=False)
            done += n
            part += 1
            _, top1 = test(teacher, dev, F.cross_entropy, val, verbose=0, shard=True)
        disable_native_convs([m for m in teacher.modules() if "forward" in m.__dict__])
    sync = pdist.sync_module(teacher)
    state = {k: v.detach().clone() for k, v in teacher.state_dict().items()}
    del teacher, opt
    t_teacher = time.perf_counter() - t0
    res = {"teacher_top1": round(top1, 4), "teacher_steps": done, "teacher_s": round(t_teacher, 1),
           "teacher_agreed_before_broadcast": sync["agreed_before"]}
    rng = np.random.RandomState(seed * 7919 + 17)
    for method in ("taylor", "random"):
        torch.manual_seed(seed)
        model = resnet50(num_classes=cfg["classes"]).to(dev).to(memory_format=torch.channels_last)
        model.load_state_dict(state)
        enable_native_convs(model)
        wrapper = PrunableDDP(model, device=dev)
        opt = _sgd(model.parameters(), cfg["ft_lr"], dev)
        pruner = Pruner(model, shape, dev, optimizer=opt)
        model.eval()
        graph = get_resnet_pruning_graph(model)
        if method == "random":
            scores = [rng.random_sample(m.out_channels) for m, _ in graph]
        else:
            data = task.stream(cfg["score_batches"] * world, cfg["batch"], seed=seed * 1000 + 200, channels_last=True)
            scores = TaylorAttributionMetric(model, data, F.cross_entropy, dev).run_many(
                [m for m, _ in graph], find_best_evaluation_module=True)
        _prune_all(model, pruner, scores, cfg["frac"])
        wrapper.rewrap()
        recalibrate_bn(model, task.stream(cfg["recal_batches"], cfg["batch"], seed=seed * 1000 + 300,
                                          channels_last=True))
        _, after_prune = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        train(wrapper, dev, F.cross_entropy, task.stream(cfg["ft_steps"] * world, cfg["batch"],
                                                         seed=seed * 1000 + 100, channels_last=True), opt, 0,
              log_every=0)
        _, after_ft = test(model, dev, F.cross_entropy, val, verbose=0, shard=True)
        res[f"{method}_after_prune"] = round(after_prune, 4)
        res[f"{method}_after_finetune"] = round(after_ft, 4)
        res["params_after"] = count_parameters(model)
        res[f"{method}_in_sync"] = params_in_sync(model)
        disable_native_convs([m for m in model.modules() if "forward" in m.__dict__])
        del model, wrapper, opt, pruner
    res["config"] = {k: cfg[k] for k in ("res", "classes", "modes", "noise", "label_noise", "batch", "frac",
                                         "ft_steps", "lr", "ft_lr", "recal_batches", "teacher_target")}
    res["note"] = "finetune batches are per GPU (weak scaling): the finetuned top-1 depends on the rank count"
    return res
