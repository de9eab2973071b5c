#!/usr/bin/env python
"""Attribution comparison on the toy 2-4-1 "max" network (reference notebook nbMAX:17-93).

Hand-set weights realise y = max(x1, x2); unit D has an extra outgoing edge (version 2). On
100 random inputs the notebook compares gradient (Sensitivity), Taylor and Shapley values
(nbMAX:43-48). Here every method of the library is evaluated through the public API.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, TensorDataset

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric,  # noqa: E402
                             ShapleyAttributionMetric, TaylorAttributionMetric, WeightNormAttributionMetric)


def max_model(w_d=-0.1):
    w1 = torch.tensor([[-0.5, 1.0, 1.0, 1.0], [0.5, -1.0, 1.0, 1.0]]).float()
    w2 = torch.tensor([[1], [0.5], [0.5], [w_d]]).float()
    l1, l2 = nn.Linear(2, 4, bias=False), nn.Linear(4, 1, bias=False)
    l1.weight.data, l2.weight.data = w1.t().contiguous(), w2.t().contiguous()
    return nn.Sequential(l1, nn.ReLU(), l2)


def main():
    torch.manual_seed(0)
    np.random.seed(0)
    model = max_model()
    x = torch.rand(100, 2) * 2
    y = x.max(1, keepdim=True).values
    dl = DataLoader(TensorDataset(x, y), batch_size=1, shuffle=False)
    dev = torch.device("cpu")
    res = {}
    for name, m in [("weight_norm", WeightNormAttributionMetric(model, dl, F.mse_loss, dev)),
                    ("apoz", APoZAttributionMetric(model, dl, F.mse_loss, dev)),
                    ("gradient", SensitivityAttributionMetric(model, dl, F.mse_loss, dev)),
                    ("taylor_signed", TaylorAttributionMetric(model, dl, F.mse_loss, dev, signed=True)),
                    ("shapley", ShapleyAttributionMetric(model, dl, F.mse_loss, dev, sv_samples=100))]:
        res[name] = [round(float(v), 4) for v in m.run(model[0])]
    res["reference_notebook"] = {"gradient": [4.01, 1.00, 1.00, 0.20], "taylor": [-1.70, -1.62, -11.72, 2.34],
                                 "sv": [0.80, 0.76, 4.96, -1.04],
                                 "note": "nbMAX:43-48, different random points / loss scaling (stale outputs)"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
