"""Calibrate the headline accuracy protocol (bench/prune_quality.py) for an unsaturated teacher.

For every noise level, runs the full protocol (teacher -> Taylor- and Random-pruned copies) over
several seeds and prints one JSON line per run plus a summary per noise level: teacher top-1
mean, Taylor / Random top-1 mean +- std, the paired Taylor - Random difference and its sign
count. Usage: python scripts/probes/quality_calib.py --noise 3.5 4.0 --seeds 0 1 2 3 4 [--teacher-steps N]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd.bench import prune_quality as pq  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--noise", type=float, nargs="+", default=[3.5, 4.0])
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--teacher-steps", type=int, default=None)
    ap.add_argument("--modes", type=int, default=None)
    ap.add_argument("--label-noise", type=float, default=None)
    ap.add_argument("--set", nargs="*", default=[], help="extra protocol overrides key=value (numbers)")
    args = ap.parse_args()
    for noise in args.noise:
        over = {"noise": noise}
        if args.teacher_steps:
            over["teacher_steps"] = args.teacher_steps
        if args.modes:
            over["modes"] = args.modes
        if args.label_noise is not None:
            over["label_noise"] = args.label_noise
        for kv in args.set:
            k, v = kv.split("=")
            over[k] = float(v) if "." in v or "e" in v else int(v)
        runs = []
        for s in args.seeds:
            r = pq.run_protocol(s, "cuda", **over)
            r.pop("config", None)
            print(json.dumps(dict(r, noise=noise)), flush=True)
            runs.append(r)
        b = np.array([r["top1_before"] for r in runs])
        t = np.array([r["top1_pruned_taylor"] for r in runs])
        rr = np.array([r["top1_pruned_random"] for r in runs])
        d = t - rr
        print(json.dumps({"summary": over, "teacher": [round(b.mean(), 4), round(b.std(), 4)],
                          "taylor": [round(t.mean(), 4), round(t.std(), 4)],
                          "random": [round(rr.mean(), 4), round(rr.std(), 4)],
                          "diff": [round(d.mean(), 4), round(d.std(), 4)], "taylor_wins": int((d > 0).sum()),
                          "seeds": len(runs)}), flush=True)


if __name__ == "__main__":
    main()
