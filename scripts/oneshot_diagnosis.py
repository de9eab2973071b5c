"""Why does one-shot Taylor pruning (every conv at once, no finetune) lose to Random in the bench's
quality protocol (bench/prune_quality.py oneshot_prune)? Per teacher seed:

1. engine vs an independent plain-PyTorch (MIOpen, autograd hooks) implementation of the
   reference Taylor formula (taylor.py:38-49: -(g * a) summed over space, |.| per sample, mean over
   samples) on the same teacher and images: per-layer Spearman and max relative difference;
2. one-shot top-1 at 30 / 50 % for several criteria: engine Taylor, PyTorch Taylor, Random, APoZ,
   weight norm, Sensitivity, and Taylor inverted (prune the HIGHEST scores: a ranking that carries
   signal must do far worse inverted);
3. the same with only ONE layer pruned at a time (the per-layer ranking quality in isolation).

python scripts/oneshot_diagnosis.py [--seeds 0 1] [--out profiles/quality/oneshot_diagnosis_r5.json]"""
import argparse
import copy
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spearman(a, b):
    ra = np.argsort(np.argsort(a)).astype(np.float64)
    rb = np.argsort(np.argsort(b)).astype(np.float64)
    ra -= ra.mean()
    rb -= rb.mean()
    return float((ra * rb).sum() / np.sqrt((ra * ra).sum() * (rb * rb).sum()))


def torch_taylor(model, convs, xs, ys, batch=100):
    """Reference formula, independent implementation: hooks on the ReLU after each conv's BN."""
    from torchpruner_amd.utils import find_best_module_for_attributions
    mods = [find_best_module_for_attributions(model, c) for c in convs]
    acc = [[] for _ in mods]
    saved = {}

    def fwd(i):
        def hook(_m, _inp, out):
            saved[i] = out

            def bwd(g):
                t = (-(g * saved[i])).flatten(2).sum(-1).abs()
                acc[i].append(t.detach().double().cpu())
            out.register_hook(bwd)
        return hook

    hs = [m.register_forward_hook(fwd(i)) for i, m in enumerate(mods)]
    model.eval()
    try:
        for s in range(0, xs.shape[0], batch):
            model.zero_grad(set_to_none=True)
            F.cross_entropy(model(xs[s:s + batch]), ys[s:s + batch]).backward()
    finally:
        for h in hs:
            h.remove()
    model.zero_grad(set_to_none=True)
    return [torch.cat(a).mean(0).numpy() for a in acc]


def scores_for(method, model, convs, xs, ys, dev, seed, frac):
    from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, TaylorAttributionMetric,
                                 WeightNormAttributionMetric)
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine.fused_chain import TUNER
    cls = {"taylor": TaylorAttributionMetric, "taylor_inverted": TaylorAttributionMetric,
           "apoz": APoZAttributionMetric, "sensitivity": SensitivityAttributionMetric,
           "weight_norm": WeightNormAttributionMetric}
    if method == "random":
        rng = np.random.RandomState(seed * 31 + int(frac * 100))
        return [rng.random_sample(m.out_channels) for m in convs]
    if method == "taylor_torch":
        return torch_taylor(model, convs, xs, ys)
    model.eval()
    with TUNER.fixed():
        s = cls[method](model, DeviceLoader(xs, ys, 100), F.cross_entropy, dev,
                        shard_data=False).run_many(convs, find_best_evaluation_module=True)
    return [-np.asarray(v) for v in s] if method == "taylor_inverted" else s


def prune_with(model, graph, scores, frac, only=None):
    from torchpruner_amd import Pruner
    dev = next(model.parameters()).device
    pruner = Pruner(model, (3, 32, 32), dev, sync_indices=False)
    for li, ((module, cascade), s) in enumerate(zip(graph, scores)):
        if only is not None and li != only:
            continue
        cut = int(len(s) * frac)
        if cut > 0:
            pruner.prune_model(module, np.argsort(s, kind="stable")[:cut], cascading_modules=cascade)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--out", default="")
    ap.add_argument("--per-layer", action="store_true", help="also prune one layer at a time (13 x methods runs)")
    args = ap.parse_args()
    from torchpruner_amd.bench.prune_quality import (DEFAULTS, ONESHOT_RECAL, make_teacher, recalibrate, top1)
    from torchpruner_amd.utils import get_vgg_pruning_graph
    dev = torch.device("cuda")
    methods = ["taylor", "taylor_torch", "random", "apoz", "weight_norm", "sensitivity", "taylor_inverted"]
    report = {"methods": methods, "seeds": {}}
    for seed in args.seeds:
        cfg = dict(DEFAULTS)
        teacher, task = make_teacher(seed, dev, cfg)
        xv, yv = task.sample(cfg["val_imgs"], seed * 7 + 3)
        xs, ys = task.sample(cfg["score_imgs"], seed * 7 + 11)
        rec = {"before": top1(teacher, xv, yv)}
        graph = [(m, c) for m, c in get_vgg_pruning_graph(teacher) if isinstance(m, torch.nn.Conv2d)]
        convs = [m for m, _ in graph]
        sc = {m: scores_for(m, teacher, convs, xs, ys, dev, seed, 0.5) for m in methods if m != "random"}
        rec["engine_vs_torch_taylor"] = [
            {"spearman": round(spearman(a, b), 6),
             "max_rel_diff": float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))}
            for a, b in zip(sc["taylor"], sc["taylor_torch"])]
        # how concentrated are Taylor's lowest-half units: fraction of near-dead units per layer
        rec["taylor_zero_frac"] = [float((np.asarray(s) <= 1e-12).mean()) for s in sc["taylor"]]
        for frac in (0.3, 0.5):
            for m in methods:
                s = scores_for(m, teacher, convs, xs, ys, dev, seed, frac) if m == "random" else sc[m]
                model = copy.deepcopy(teacher)
                g2 = [(dict(model.named_modules())[n], [dict(model.named_modules())[k] for k in ks])
                      for n, ks in _graph_names(teacher, graph)]
                prune_with(model, g2, s, frac)
                recalibrate(model, task, seed * 1000 + 777, dict(cfg, recal_batches=ONESHOT_RECAL))
                rec[f"oneshot_{int(frac * 100)}_{m}"] = top1(model, xv, yv)
                del model
            print(f"seed {seed} frac {frac}: " + ", ".join(f"{m} {rec[f'oneshot_{int(frac * 100)}_{m}']:.4f}"
                                                           for m in methods), flush=True)
        if args.per_layer:
            for m in ("taylor", "random", "weight_norm"):
                row = []
                for li in range(len(graph)):
                    s = scores_for(m, teacher, convs, xs, ys, dev, seed, 0.5) if m == "random" else sc[m]
                    model = copy.deepcopy(teacher)
                    g2 = [(dict(model.named_modules())[n], [dict(model.named_modules())[k] for k in ks])
                          for n, ks in _graph_names(teacher, graph)]
                    prune_with(model, g2, s, 0.5, only=li)
                    recalibrate(model, task, seed * 1000 + 777, dict(cfg, recal_batches=ONESHOT_RECAL))
                    row.append(top1(model, xv, yv))
                    del model
                rec[f"single_layer_50_{m}"] = row
                print(f"seed {seed} single-layer 50% {m}: {[round(v, 3) for v in row]}", flush=True)
        print(f"seed {seed}: engine vs torch Taylor spearman min "
              f"{min(r['spearman'] for r in rec['engine_vs_torch_taylor']):.6f}", flush=True)
        report["seeds"][str(seed)] = rec
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)


def _graph_names(model, graph):
    names = {id(m): n for n, m in model.named_modules()}
    return [(names[id(m)], [names[id(c)] for c in cas]) for m, cas in graph]


if __name__ == "__main__":
    main()
