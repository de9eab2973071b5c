"""The round-6 bench additions on the GPU (small shapes: reporting paths, not the numbers):
``vgg_taylor_pruned50_img_s`` (the headline workload on the network a 50 % prune produces) and the
layerwise ablation AUC of the accuracy half (nbVGG:1233-1285, 1521-1527), checked against a plain
PyTorch re-implementation of the notebook's loop for one layer."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(260)
def test_bench_pruned_extra(cuda):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONUNBUFFERED"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch",
                        "128", "--teacher-steps", "20", "--no-baseline", "--no-prune", "--extras", "pruned"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["vgg_taylor_pruned50_img_s"] > 0 and out["pruned50_vs_dense"] > 0
    cfg = out["pruned50_config"]
    assert cfg["widths"] == [32, 32, 64, 64, 128, 128, 128, 256, 256, 256, 256, 256, 256]
    assert 0.2 < cfg["conv_mac_fraction"] < 0.3  # half of every conv: ~1/4 of the MACs
    assert cfg["tuner_choices"], cfg


def test_layerwise_auc_matches_notebook_loop(cuda):
    """prune_quality.layerwise_auc == the reference notebook's sequential index_fill_ loop (one
    forward per removed unit, nbVGG:1265-1280) for the Random ranking of one layer, and sane output
    for every method."""
    from torchpruner_amd.bench import prune_quality as pq
    from torchpruner_amd.utils import find_best_module_for_attributions
    cfg = dict(pq.DEFAULTS, teacher_steps=60)
    model, task = pq.make_teacher(0, cuda, cfg)
    lw = dict(attr_imgs=200, ablation_imgs=200, sv_samples=2, random_draws=1)
    out = pq.layerwise_auc(model, task, 0, lw=lw)
    for m in ("taylor", "random", "sv"):
        assert np.isfinite(out[f"layerwise_auc_{m}"]), out
        assert len(out[f"layerwise_auc_{m}_per_layer"]) == 13
    # notebook loop for the last conv's Random ranking (same draw as layerwise_auc's first one)
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    rng = np.random.RandomState(0 * 17 + 3)
    draws = [rng.random_sample(c.out_channels) for c in convs]
    xt, yt = task.sample(lw["ablation_imgs"], 0 * 7 + 102)
    k = len(convs) - 1
    ev = find_best_module_for_attributions(model, convs[k])
    model.eval()
    with torch.no_grad():
        z = model.forward_partial(xt, to_module=ev).clone()
        base = float(F.cross_entropy(model.forward_partial(z, from_module=ev), yt))
        inc = 0.0
        for i in np.argsort(draws[k], kind="stable"):
            z.index_fill_(1, torch.tensor([int(i)], device=z.device), 0.0)
            inc += float(F.cross_entropy(model.forward_partial(z, from_module=ev), yt)) - base
    ref = inc / convs[k].out_channels
    got = out["layerwise_auc_random_per_layer"][k]
    assert abs(got - ref) <= 1e-3 * max(1.0, abs(ref)), (got, ref)
