"""Calibrate config #5's prune -> finetune round (bench/resnet_finetune.QUALITY) on one GPU.

Runs prune_finetune_quality for every combination of the given overrides and prints one JSON line
per run (teacher top-1, Taylor / Random after prune and after finetune).
Usage: python scripts/probes/config5_calib.py --set lr=0.01,0.003 ft_steps=15,60 --seeds 0 1
"""
import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from torchpruner_amd.bench import resnet_finetune as rf  # noqa: E402


def _num(v):
    return float(v) if "." in v or "e" in v else int(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", nargs="*", default=[], help="key=v1,v2,... (the grid is their product)")
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    args = ap.parse_args()
    keys, vals = [], []
    for kv in args.set:
        k, v = kv.split("=")
        keys.append(k)
        vals.append([_num(x) for x in v.split(",")])
    dev = torch.device("cuda")
    for combo in itertools.product(*vals) if vals else [()]:
        cfg = dict(zip(keys, combo))
        for s in args.seeds:
            r = rf.prune_finetune_quality(dev, 1, 0, seed=s, cfg=cfg)
            r.pop("config", None)
            print(json.dumps(dict(cfg, seed=s, **r)), flush=True)


if __name__ == "__main__":
    main()
