"""Same teacher, three Taylor implementations (engine+Winograd, engine direct-GEMM, generic
hook path with MIOpen): rank agreement and the layerwise 50% top-1 of each, plus Random over
several seeds."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torchpruner_amd.attributions import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.data import DeviceLoader, PrototypeTask  # noqa: E402
from torchpruner_amd.engine import fused_chain as fc  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.parallel import dist as pdist  # noqa: E402

steps = int(os.environ.get("TEACHER_STEPS", "150"))
noise = float(os.environ.get("NOISE", "2.0"))
tseed = int(os.environ.get("TSEED", "0"))
modes = int(os.environ.get("MODES", "1"))
pdist.init_distributed()
dev = torch.device("cuda")
torch.manual_seed(tseed)
model = prunable_vgg16().to(dev)
task = PrototypeTask((3, 32, 32), 10, noise=noise, seed=tseed, device=dev, modes_per_class=modes)
bench.train_teacher(model, task, steps, dev, tseed)
convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
xt, yt = task.sample(10 * 512, 2)
xv, yv = task.sample(2000, 3)
print(f"noise {noise} modes {modes} tseed {tseed} steps {steps}: top1 before", bench.top1(model, xv, yv), "train-set top1", bench.top1(model, xt[:2000], yt[:2000]))


def scores(tag):
    fc._ENGINES.clear()
    fc.TUNER.cache.clear()
    m = TaylorAttributionMetric(model, DeviceLoader(xt, yt, 512), F.cross_entropy, dev)
    return m.run_many(convs, find_best_evaluation_module=True)


res = {}
os.environ["TORCHPRUNER_WINOGRAD"] = "1"
res["wino"] = scores("wino")
os.environ["TORCHPRUNER_WINOGRAD"] = "0"
res["direct"] = scores("direct")
os.environ["TORCHPRUNER_BACKEND"] = "torch"
res["hook"] = scores("hook")
os.environ.pop("TORCHPRUNER_BACKEND")
for k, s in res.items():
    agree = [np.mean(np.sort(np.argsort(a)[: len(a) // 2]) == np.sort(np.argsort(b)[: len(b) // 2]))
             for a, b in zip(s, res["hook"])]
    rel = [float(np.linalg.norm(a - b) / np.linalg.norm(b)) for a, b in zip(s, res["hook"])]
    print(f"{k:7s} layerwise50 {bench.layerwise_top1(model, convs, s, xv, yv):.4f}  "
          f"bottom-half set agreement vs hook {np.mean(agree):.3f}  max rel diff {max(rel):.2e}")
for seed in range(3):
    rng = np.random.RandomState(seed)
    print(f"random{seed} layerwise50 "
          f"{bench.layerwise_top1(model, convs, [rng.random_sample(c.out_channels) for c in convs], xv, yv):.4f}")
per = [bench.layerwise_top1(model, [c], [s], xv, yv) for c, s in zip(convs, res["wino"])]
print("per-layer wino:", " ".join(f"{p:.2f}" for p in per))
