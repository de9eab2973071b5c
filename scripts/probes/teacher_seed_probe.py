"""The bench's VGG16 teacher (bench/prune_quality.make_teacher) for a few seeds: top-1 on the
held-out split, with the training weight-pack cache on and off (TORCHPRUNER_BATCH_WEIGHT_PACK
semantics via engine.train._BATCH_PACK). python scripts/probes/teacher_seed_probe.py [seeds...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchpruner_amd.bench import prune_quality as pq  # noqa: E402
from torchpruner_amd.engine import train as tr  # noqa: E402

seeds = [int(s) for s in sys.argv[1:]] or [0, 1]
for batch_pack in (True, False):
    tr._BATCH_PACK = batch_pack
    for seed in seeds:
        cfg = dict(pq.DEFAULTS)
        model, task = pq.make_teacher(seed, torch.device("cuda"), cfg)
        xv, yv = task.sample(cfg["val_imgs"], seed * 7 + 3)
        print(f"batch_pack={batch_pack} seed {seed}: top-1 {pq.top1(model, xv, yv):.4f}", flush=True)
        del model
