"""F(4x4,3x3): the WIDE kernel (variant 1: 64-tile blocks, one wave per SIMD, 32 outputs per wave)
vs the MODE 3 kernel (variant 0: 32-tile blocks, two blocks per CU) on the VGG16-CIFAR conv
shapes: per-layer us for the forward (BN+ReLU, pooled where VGG pools) and the data gradient
(Taylor partials), each at its best split count, plus the max relative difference of the two.

    python scripts/probes/wino4_wide_bench.py [--batch 2048] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

LAYERS = [(32, 64, 64, True), (16, 64, 128, False), (16, 128, 128, True), (8, 128, 256, False),
          (8, 256, 256, False), (8, 256, 256, True), (4, 256, 512, False), (4, 512, 512, False),
          (4, 512, 512, True)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def splits_for(B, S, K, C, tb, per_cu):
    blocks = -(-B * (S // 4) ** 2 // tb) * (K // 32)
    out, sp = [1], 1
    while blocks * sp < per_cu * 256 and sp * 2 <= (C // 8) // 4 and sp < 16:
        sp *= 2
        out.append(sp)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[2048, 100])
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    for B in args.batch:
        tot = {"f0": 0.0, "f1": 0.0, "b0": 0.0, "b1": 0.0}
        print(f"B={B}: per layer us, best split (MODE 3 -> WIDE), max rel diff", flush=True)
        for S, C, K, pool in LAYERS:
            g = torch.Generator(device=dev).manual_seed(S + C + K)
            x = torch.randn(B, S, S, C, device=dev, generator=g)
            w = torch.randn(K, C, 3, 3, device=dev, generator=g) * 0.05
            sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
            u4 = T.wino4_weights(w, False, 0, 0)
            res = {}
            for var, tb, per_cu in ((0, 32, 2), (1, 64, 1)):
                best = None
                for sp in splits_for(B, S, K, C, tb, per_cu):
                    t = timeit(lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None, sp, var), args.iters)
                    if best is None or t < best[0]:
                        best = (t, sp)
                res[("f", var)] = best
            y0, _ = T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None, 1, 0)
            y1, _ = T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None, 1, 1)
            dfw = ((y0 - y1).abs().max() / y0.abs().max()).item()
            gg = torch.randn(B, S, S, K, device=dev, generator=g)
            act = torch.relu(torch.randn(B, S, S, C, device=dev, generator=g))
            scp = torch.rand(C, device=dev) + 0.5
            ut4 = T.wino4_weights(w, True, 0, 0)
            tay = torch.zeros(4, B, C, device=dev)
            if C % 32 == 0:
                for var, tb, per_cu in ((0, 32, 2), (1, 64, 1)):
                    best = None
                    for sp in splits_for(B, S, C, K, tb, per_cu):
                        t = timeit(lambda: T.conv_wino4_dgrad(gg, ut4, act, scp, tay, True, 0, sp, var), args.iters)
                        if best is None or t < best[0]:
                            best = (t, sp)
                    res[("b", var)] = best
                o0 = T.conv_wino4_dgrad(gg, ut4, act, scp, None, True, 0, 1, 0)
                o1 = T.conv_wino4_dgrad(gg, ut4, act, scp, None, True, 0, 1, 1)
                dbw = ((o0 - o1).abs().max() / o0.abs().max()).item()
            else:
                res[("b", 0)] = res[("b", 1)] = (float("nan"), 0)
                dbw = float("nan")
            for k in ("f", "b"):
                for v in (0, 1):
                    tot[f"{k}{v}"] += res[(k, v)][0]
            print(f"S={S:2d} C={C:3d} K={K:3d} pool={int(pool)} | fwd {res[('f', 0)][0]:7.1f} (sp{res[('f', 0)][1]}) -> "
                  f"{res[('f', 1)][0]:7.1f} (sp{res[('f', 1)][1]}) x{res[('f', 0)][0] / res[('f', 1)][0]:4.2f} "
                  f"[{dfw:.1e}] | dgrad {res[('b', 0)][0]:7.1f} (sp{res[('b', 0)][1]}) -> {res[('b', 1)][0]:7.1f} "
                  f"(sp{res[('b', 1)][1]}) x{res[('b', 0)][0] / res[('b', 1)][0]:4.2f} [{dbw:.1e}]", flush=True)
        print(f"total fwd {tot['f0']:.0f} -> {tot['f1']:.0f} us (x{tot['f0'] / tot['f1']:.2f}); dgrad {tot['b0']:.0f} "
              f"-> {tot['b1']:.0f} us (x{tot['b0'] / tot['b1']:.2f})", flush=True)


if __name__ == "__main__":
    main()
