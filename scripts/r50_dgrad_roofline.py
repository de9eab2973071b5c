"""Per-shape roofline of the ResNet-50 1x1 data gradients of the Taylor / Sensitivity engine
(B=256, fp32): for every stride-1 1x1 bottleneck conv Cin -> Cout at H x W, the dgrad GEMM
(M = B*H*W, N = Cin, K = Cout) with the ReLU-backward mask (the conv input's activation) and, for
a block's conv1, the residual gradient, timed over every candidate of the engine
(ResNetEngine._dgrad: implicit-GEMM tile configs x split-K). Bytes = g + mask + out (+ res) +
weights; roofline = max(FLOP / 155 TF, bytes / 5.5 TB/s).
Usage: python scripts/r50_dgrad_roofline.py [--batch 256] [--iters 10] [--verbose]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import TUNER  # noqa: E402

PEAK_TF, PEAK_TBS = 155.0, 5.5

# (Cin, Cout, H, count, conv1-with-residual) of the stride-1 1x1 convs of torchvision ResNet-50
SHAPES = [(64, 64, 56, 1, True), (256, 64, 56, 2, True), (64, 256, 56, 3, False),
          (512, 128, 28, 3, True), (128, 512, 28, 4, False),
          (1024, 256, 14, 5, True), (256, 1024, 14, 6, False),
          (2048, 512, 7, 2, True), (512, 2048, 7, 3, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()
    T = ops.require()
    dev = torch.device("cuda")
    B = args.batch
    tot, roof_tot = 0.0, 0.0
    print(f"{'cin':>5} {'cout':>5} {'hw':>4} {'n':>2} {'res':>3} {'best':>10} {'us':>8} {'TF/s':>6} {'TB/s':>6} {'roof%':>6}")
    for cin, cout, H, n, with_res in SHAPES:
        M = B * H * H
        g = torch.randn(B, H, H, cout, device=dev)
        wt = torch.randn(cin, cout, device=dev) * 0.05  # dgrad operand (N = cin, K = cout)
        mask = torch.randn(B, H, H, cin, device=dev).clamp_min(0)
        res = torch.randn(B, H, H, cin, device=dev) if with_res else None
        results = []
        for cfg, sp in TUNER.candidates(M, cin, cout):
            def run():
                return T.conv_gen_bwd(g, wt, res, 1, mask, 1, 1, 0, 0, 0, False, cfg, sp)
            try:
                run()
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            results.append((e0.elapsed_time(e1) / args.iters * 1e3, cfg, sp))
        us, cfg, sp = min(results)
        if args.verbose:
            print("   " + "  ".join(f"{c}/{p_}:{t:.0f}" for t, c, p_ in sorted(results, key=lambda r: (r[1], r[2]))))
        flop = 2.0 * M * cin * cout
        byts = 4.0 * (M * cout + M * cin * (3 if with_res else 2) + cin * cout)
        roof = max(flop / (PEAK_TF * 1e12), byts / (PEAK_TBS * 1e12)) * 1e6
        tot += us * n
        roof_tot += roof * n
        print(f"{cin:>5} {cout:>5} {H:>4} {n:>2} {int(with_res):>3} {f'igemm{cfg} sp{sp}':>10} {us:>8.1f} "
              f"{flop / us / 1e6:>6.1f} {byts / us / 1e6:>6.2f} {100 * roof / us:>5.0f}%", flush=True)
    print(f"sum (x count): {tot / 1e3:.2f} ms, roofline {roof_tot / 1e3:.2f} ms ({100 * roof_tot / tot:.0f}%)")


if __name__ == "__main__":
    main()
