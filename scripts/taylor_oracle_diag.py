"""Per-kernel-family error of the fused VGG16 Taylor scores against fp64.

Inputs: test_engine_taylor_matches_generic_path's (seed 0, 48 images, B=16). For each pinned
kernel family (engine.fused_chain.family_policy) and the timed / fixed tuner, prints per block:
  plain  - relative max error of the reduced scores vs the plain fp64 run (the test's oracle)
  cond   - the same vs the fp64 run that replays the engine's own ReLU masks / pool argmaxes
  flips  - units whose mask or argmax differs between the engine and plain fp64
Usage: python scripts/taylor_oracle_diag.py [--out gpurun_out/taylor_oracle.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchpruner_amd import TaylorAttributionMetric  # noqa: E402
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.engine import maybe_engine  # noqa: E402
from torchpruner_amd.engine.fused_chain import TUNER, family_policy  # noqa: E402
from torchpruner_amd.engine.oracle import engine_scores_fp64  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.utils import find_best_module_for_attributions  # noqa: E402


def reduce(per_sample, signed, red):
    s = per_sample if signed else np.abs(per_sample)
    return s.mean(0) if red == "mean" else s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/taylor_oracle.json")
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    lins = [model.classifier[1], model.classifier[4]]
    x = torch.randn(48, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (48,), device=dev)
    mods = convs + lins
    ev = [find_best_module_for_attributions(model, m) for m in mods]
    eng, idx = maybe_engine(model, ev, F.cross_entropy, dev)
    B = args.batch
    nb = x.shape[0] // B
    # fp64 references per batch (the plain one does not depend on the engine's kernels)
    policies = [("tuned", None), ("fixed", "fixed")] + [(f"{f}/{s}", (f, s)) for f in
                                                       ("wino4", "wino2", "wino2_direct", "igemm")
                                                       for s in ("min", "max")]
    rows = {}
    plain = None
    for name, pol in policies:
        ctx = TUNER.fixed() if pol == "fixed" else (TUNER.pinned(family_policy(*pol)) if pol else None)
        if ctx is not None:
            ctx.__enter__()
        try:
            fused, cond, flips = {b: [] for b in idx}, {b: [] for b in idx}, {b: 0 for b in idx}
            plain_b = {b: [] for b in idx}
            for i in range(nb):
                xb, yb = x[i * B:(i + 1) * B], y[i * B:(i + 1) * B]
                res = eng.taylor(xb, yb, set(idx))
                for b in idx:
                    t = res[b]
                    t = t.sum(0) if t.dim() == 3 else t
                    fused[b].append(t[:, :eng.real_width(b)].double().cpu())
                sc, fl = engine_scores_fp64(eng, xb, yb, conditioned=True)
                for b in idx:
                    cond[b].append(sc[b])
                    flips[b] += fl[b]
                if plain is None:
                    sp, _ = engine_scores_fp64(eng, xb, yb, conditioned=False)
                    for b in idx:
                        plain_b[b].append(sp[b])
            if plain is None:
                plain = {b: torch.cat(v).numpy() for b, v in plain_b.items()}
            # the public API under the same pinned choices (must equal the direct engine scores)
            api = TaylorAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, dev).run_many(mods, True)
            choices = {str(k): list(v) for k, v in TUNER.cache.items()}
        finally:
            if ctx is not None:
                ctx.__exit__(None, None, None)
        table = []
        for li, b in enumerate(idx):
            f = torch.cat(fused[b]).numpy()
            c = torch.cat(cond[b]).numpy()
            row = {"block": b, "flips": flips[b]}
            for signed in (False, True):
                for red in ("mean", "none"):
                    e = reduce(plain[b], signed, red)
                    scale = np.abs(e).max() + 1e-30
                    tag = f"{'s' if signed else 'u'}_{red}"
                    row[f"plain_{tag}"] = float(np.abs(reduce(f, signed, red) - e).max() / scale)
                    ec = reduce(c, signed, red)
                    row[f"cond_{tag}"] = float(np.abs(reduce(f, signed, red) - ec).max() / (np.abs(ec).max() + 1e-30))
            row["api_vs_direct"] = float(np.abs(api[li] - reduce(f, False, "mean")).max() /
                                         (np.abs(reduce(f, False, "mean")).max() + 1e-30))
            table.append(row)
        rows[name] = {"table": table, "choices": choices}
        print(f"== {name}")
        print(" blk flips  plain_u_mean cond_u_mean  plain_u_none cond_u_none  plain_s_mean cond_s_mean  api")
        for r in table:
            print(f" {r['block']:3d} {r['flips']:5d}  {r['plain_u_mean']:.2e}    {r['cond_u_mean']:.2e}     "
                  f"{r['plain_u_none']:.2e}    {r['cond_u_none']:.2e}     {r['plain_s_mean']:.2e}    "
                  f"{r['cond_s_mean']:.2e}   {r['api_vs_direct']:.1e}", flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
