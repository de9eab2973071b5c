"""Config #1: 2-layer MLP on MNIST-shaped data, WeightNormAttributionMetric + prune_model 10% of
every hidden layer, on CPU (plumbing check, no GPU).

    python -m torchpruner_amd.bench.mlp_weightnorm [--device cpu] [--frac 0.1]

Reference semantics: ``WeightNormAttributionMetric.run`` (reference methods/weight_norm.py:5-23)
scores each hidden unit by the L1 norm of its incoming weights; ``Pruner.prune_model``
(reference pruner/pruner.py:21-57) removes the lowest 10% and cascades the cut through the next
Linear (the NaN-probe discovers the consumer). The pruned model must still run and its
state_dict keeps the reference's keys with smaller shapes. Synthetic data: the scores do not
depend on data, the accuracy check uses a synthetic prototype task.
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import Pruner, WeightNormAttributionMetric
from torchpruner_amd.data import DeviceLoader, PrototypeTask
from torchpruner_amd.models import mnist_fc
from torchpruner_amd.utils import count_parameters, get_vgg_pruning_graph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--frac", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device(args.device)
    torch.manual_seed(args.seed)
    model = mnist_fc().to(dev).eval()
    task = PrototypeTask((1, 28, 28), 10, noise=1.0, seed=args.seed, device=dev)
    x, y = task.sample(1000, args.seed)
    loader = DeviceLoader(x, y, 100)
    params0 = count_parameters(model)
    sd_keys = list(model.state_dict().keys())
    t0 = time.perf_counter()
    pruner = Pruner(model, (1, 28, 28), dev)
    pruned = {}
    names = {m: n for n, m in model.named_modules()}
    for module, cascade in get_vgg_pruning_graph(model):  # last layer first, final classifier excluded
        scores = WeightNormAttributionMetric(model, loader, F.cross_entropy, dev).run(module)
        idx = np.argsort(scores, kind="stable")[: int(len(scores) * args.frac)]
        pruner.prune_model(module, idx, cascading_modules=cascade)
        pruned[names[module]] = len(idx)
    dt = time.perf_counter() - t0
    with torch.no_grad():
        out = model(x)
    assert list(model.state_dict().keys()) == sd_keys  # format preserved, shapes shrink
    res = {
        "config": "#1 MLP MNIST-shape WeightNorm prune 10% (CPU plumbing)",
        "device": str(dev),
        "params_before": params0,
        "params_after": count_parameters(model),
        "units_pruned": pruned,
        "seconds": round(dt, 4),
        "output_shape": list(out.shape),
        "hidden_widths": [m.out_features for m in model.modules() if isinstance(m, nn.Linear)][:-1],
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
