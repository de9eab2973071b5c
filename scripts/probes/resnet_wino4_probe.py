"""ResNet-50 stride-1 3x3 convs (B=256, C=K at 56/28/14/7 px): F(2x2) staged Winograd vs the
F(4x4) split-points kernel (band geometry), forward (BN affine + ReLU + APoZ) and data gradient
(mask + Taylor partials), best channel split of each; us per launch and the F(4x4) speed-up.
python scripts/probes/resnet_wino4_probe.py [--B 256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(rounds):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    dev = torch.device("cuda")
    B = args.B
    tot = [0.0, 0.0, 0.0, 0.0]
    for S, C in ((56, 64), (28, 128), (14, 256), (7, 512)):
        x = torch.relu(torch.randn(B, S, S, C, device=dev))
        w = torch.randn(C, C, 3, 3, device=dev) / (3 * C ** 0.5)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        u2 = winograd_weights(w)
        u2t = winograd_weights(w.flip(2, 3).transpose(0, 1).contiguous())
        u4 = T.wino4_weights(w, False, 0, 0)
        u4t = T.wino4_weights(w, True, 0, 0)
        g = torch.randn(B, S, S, C, device=dev)
        ap_ = torch.zeros(B, C, device=dev)
        tay2 = torch.zeros(64, B, C, device=dev)
        tay4 = torch.zeros(T.wino4_taylor_slots(S), B, C, device=dev)
        f2 = min(timeit(lambda: T.conv_wino_fwd(x, u2, sc, sh, True, False, sp, True, ap_)) for sp in (1, 2, 4))
        f4 = min(timeit(lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, False, ap_, sp, 3)) for sp in (1, 2))
        d2 = min(timeit(lambda: T.conv_wino_dgrad(g, None, u2t, x, None, tay2, True, sp, True, 0)) for sp in (1, 2, 4))
        d4 = min(timeit(lambda: T.conv_wino4_dgrad(g, u4t, x, None, tay4, True, 0, sp, 3)) for sp in (1, 2))
        for i, v in enumerate((f2, f4, d2, d4)):
            tot[i] += v
        print(f"S={S:2d} C=K={C:3d}: fwd F(2x2) {f2:7.1f} us  F(4x4) {f4:7.1f} us  x{f2 / f4:4.2f} | "
              f"dgrad F(2x2) {d2:7.1f} us  F(4x4) {d4:7.1f} us  x{d2 / d4:4.2f}", flush=True)
    print(f"sum: fwd {tot[0]:.0f} -> {tot[1]:.0f} us, dgrad {tot[2]:.0f} -> {tot[3]:.0f} us", flush=True)


if __name__ == "__main__":
    main()
