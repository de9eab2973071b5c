"""Config #4: VGG16 / CIFAR-10 ShapleyAttributionMetric (sv_samples=5), prefix evaluations
sharded across the ranks of the job (torchrun, one process per GPU).

    python -m torchpruner_amd.bench.shapley_vgg [--layers 0,6,12] [--images 1000] [--batch 100]
    torchrun --nproc-per-node 8 -m torchpruner_amd.bench.shapley_vgg ...

Reports wall time per layer and downstream image-evaluations per second (one evaluation =
one image through the layers after the masked activation), the unit of the reference's
6 h 30 min layerwise study (~9.9 k img-evals/s on its GPU, nbVGG:1228-1229).
``--reference`` also times the reference-semantics loop (one prefix per forward, host copy
of every delta) on a subset for the same layer.
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch
import torch.nn.functional as F

from torchpruner_amd import ShapleyAttributionMetric
from torchpruner_amd.data import DeviceLoader, PrototypeTask
from torchpruner_amd.models import prunable_vgg16
from torchpruner_amd.parallel import dist as pdist


def reference_semantics_shapley(model, x, y, module_eval, S, max_units):
    """One prefix per partial forward + per-delta host copy (shapley_values.py:51-61)."""
    z0 = model.forward_partial(x, to_module=module_eval)
    base = F.cross_entropy(model.forward_partial(z0, from_module=module_eval), y, reduction="none")
    n = z0.shape[1]
    sv = np.zeros((x.shape[0], n))
    evals = 0
    for j in range(S):
        z = z0.clone()
        loss = base.clone()
        for i in np.random.permutation(n)[:max_units]:
            z.index_fill_(1, torch.tensor([i], device=x.device), 0.0)
            new = F.cross_entropy(model.forward_partial(z, from_module=module_eval), y, reduction="none")
            sv[:, i] += ((new - loss) / S).cpu().numpy()
            loss = new
            evals += x.shape[0]
    return evals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="0,6,12")
    ap.add_argument("--images", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--sv-samples", type=int, default=5)
    ap.add_argument("--reference", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--model", default="vgg16", choices=["vgg16", "resnet50"],
                    help="resnet50: ImageNet-shaped input, prunable = conv1/conv2 of every bottleneck")
    args = ap.parse_args()
    ctx = pdist.init_distributed()
    dev = ctx.device
    torch.manual_seed(0)
    np.random.seed(0)
    if args.model == "resnet50":
        from torchpruner_amd import get_resnet_pruning_graph
        from torchpruner_amd.models import resnet50
        model = resnet50().to(dev).eval()
        x = torch.randn(args.images, 3, 224, 224, device=dev)
        y = torch.randint(0, 1000, (args.images,), device=dev)
        prunable = [m for m, _ in get_resnet_pruning_graph(model)][::-1]  # input -> output order
    else:
        model = prunable_vgg16().to(dev).eval()
        task = PrototypeTask((3, 32, 32), 10, noise=2.0, seed=0, device=dev)
        x, y = task.sample(args.images, 1)
        prunable = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1],
                                                                                     model.classifier[4]]
    dl = DeviceLoader(x, y, args.batch)
    metric = ShapleyAttributionMetric(model, dl, F.cross_entropy, dev, sv_samples=args.sv_samples)
    out = {"n_gpus": ctx.world_size, "images": args.images, "batch": args.batch, "sv_samples": args.sv_samples,
           "layers": []}
    for li in [int(v) for v in args.layers.split(",")]:
        module = prunable[li]
        n = module.out_channels if isinstance(module, torch.nn.Conv2d) else module.out_features
        metric.run(module, find_best_evaluation_module=True, sv_samples=1)  # warm (autotune, allocator)
        pdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        scores = metric.run(module, find_best_evaluation_module=True)
        torch.cuda.synchronize()
        pdist.barrier()
        dt = time.perf_counter() - t0
        evals = args.sv_samples * n * args.images
        row = {"layer": li, "units": n, "seconds": round(dt, 4), "img_evals_per_s": round(evals / dt, 1),
               "finite": bool(np.isfinite(scores).all())}
        if args.reference and ctx.rank == 0:
            from torchpruner_amd.utils import find_best_module_for_attributions
            ev = find_best_module_for_attributions(model, module)
            with torch.no_grad():
                xs, ys = x[: args.batch], y[: args.batch]
                reference_semantics_shapley(model, xs, ys, ev, 1, 4)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                e = reference_semantics_shapley(model, xs, ys, ev, 1, 32)
                torch.cuda.synchronize()
                row["reference_semantics_img_evals_per_s"] = round(e / (time.perf_counter() - t1), 1)
        out["layers"].append(row)
        if ctx.rank == 0:
            print(json.dumps(row), flush=True)
    if ctx.rank == 0 and args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if ctx.world_size > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
