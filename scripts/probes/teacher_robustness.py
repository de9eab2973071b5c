"""Probe: the bench's VGG16 teacher (bench/prune_quality.make_teacher) under candidate recipes — its
held-out top-1, the single-layer 50 % mask top-1 (Taylor / Random, nbVGG protocol at one point) and
the layerwise AUC (Taylor / Random). Run it twice, with and without TP_WGRAD_COMBINE_LANES=1 (the
wgrad split-sum order, read once per process), to see which recipe's teacher does not depend on the
kernels' rounding. One JSON line per (recipe, seed).

    python scripts/probes/teacher_robustness.py --seeds 0 1 2 --recipes 'lr=0.05' 'lr=0.02,teacher_steps=2000'
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.bench import prune_quality as pq  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.engine.fused_chain import TUNER  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402


def mask50(model, convs, scores, x, y):
    accs = []
    with torch.no_grad():
        for conv, s in zip(convs, scores):
            idx = torch.as_tensor(np.argsort(s, kind="stable")[: len(s) // 2], device=x.device)
            h = find_best_module_for_attributions(model, conv).register_forward_hook(
                lambda m, i, o, idx=idx: o.index_fill(1, idx, 0.0))
            try:
                accs.append(pq.top1(model, x, y))
            finally:
                h.remove()
    return float(np.mean(accs)), float(np.min(accs))


def parse_recipe(r):
    out = {}
    for kv in filter(None, r.split(",")):
        k, v = kv.split("=")
        out[k] = type(pq.DEFAULTS[k])(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--recipes", nargs="+", default=[""])
    a = ap.parse_args()
    dev = torch.device("cuda")
    lanes = os.environ.get("TP_WGRAD_COMBINE_LANES", "default")
    for r in a.recipes:
        cfg = dict(pq.DEFAULTS, **parse_recipe(r))
        for seed in a.seeds:
            t0 = time.perf_counter()
            model, task = pq.make_teacher(seed, dev, cfg)
            xv, yv = task.sample(cfg["val_imgs"], seed * 7 + 3)
            convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
            xs, ys = task.sample(1000, seed * 7 + 101)
            with TUNER.fixed():
                tay = TaylorAttributionMetric(model, DeviceLoader(xs, ys, 100), torch.nn.functional.cross_entropy,
                                              dev, shard_data=False).run_many(convs, find_best_evaluation_module=True)
            rng = np.random.RandomState(seed)
            m_t = mask50(model, convs, tay, xv, yv)
            m_r = mask50(model, convs, [rng.random_sample(c.out_channels) for c in convs], xv, yv)
            auc = pq.layerwise_auc(model, task, seed, methods=("taylor", "random"))
            print(json.dumps({"recipe": r, "lanes": lanes, "seed": seed, "top1": pq.top1(model, xv, yv),
                              "mask50_taylor_mean_min": m_t, "mask50_random_mean_min": m_r,
                              "auc_taylor": round(auc["layerwise_auc_taylor"], 4),
                              "auc_random": round(auc["layerwise_auc_random"], 4),
                              "s": round(time.perf_counter() - t0, 1)}), flush=True)
            del model


if __name__ == "__main__":
    main()
