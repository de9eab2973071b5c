"""Per-layer timings of the VGG16/CIFAR 3x3 convs at B=2048 (forward and data gradient): fp32
F(4x4) (wino4), fp32 F(2x2) staged (wino2), bf16 F(2x2) staged (wino2-bf16: bf16 U images,
v_mfma_f32_16x16x16_bf16) and the bf16-operand implicit GEMM (igemm-bf16, cfg 256+0).
python scripts/wino_bf16_bench.py [--B 2048] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (S, C, K, pool) of VGG16's 3x3 convs after the first (the engine's layout)
LAYERS = [(32, 64, 64, True), (16, 64, 128, False), (16, 128, 128, True), (8, 128, 256, False),
          (8, 256, 256, False), (8, 256, 256, True), (4, 256, 512, False), (4, 512, 512, False),
          (4, 512, 512, True)]


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    B = args.B
    tot = {}
    print(f"{'layer':>22s} {'dir':>5s} {'wino4':>9s} {'wino2':>9s} {'wino2-bf16':>11s} {'igemm-bf16':>11s}  us")
    for S, C, K, pool in LAYERS:
        x = torch.randn(B, S, S, C, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) * (2.0 / (9 * C)) ** 0.5
        sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
        u4 = T.wino4_weights(w, False, 0, 0)
        u2 = T.wino_weights(w, False, K, C)
        ub = T.wino_weights(w, False, K, C, True)
        wg = w.permute(0, 2, 3, 1).reshape(K, 9 * C).contiguous()
        fw = {
            "wino4": lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None, 1, 0),
            "wino2": lambda: T.conv_wino_fwd(x, u2, sc, sh, True, pool, 1, True),
            "wino2-bf16": lambda: T.conv_wino_fwd(x, ub, sc, sh, True, pool, 1, True),
            "igemm-bf16": lambda: T.conv_fwd(x, wg, sc, sh, True, pool, 3, 256, 1),
        }
        row = {k: _time(f, args.iters) for k, f in fw.items()}
        for k, v in row.items():
            tot[("fwd", k)] = tot.get(("fwd", k), 0.0) + v
        print(f"{str((S, C, K, pool)):>22s} {'fwd':>5s} {row['wino4']:9.1f} {row['wino2']:9.1f} "
              f"{row['wino2-bf16']:11.1f} {row['igemm-bf16']:11.1f}", flush=True)
        # data gradient of this conv (input C channels, from K-channel gradient), Taylor partials
        g = torch.randn(B, S, S, K, device=dev)
        act = torch.relu(torch.randn(B, S, S, C, device=dev))
        bn = torch.rand(C, device=dev) + 0.5
        ut4 = T.wino4_weights(w, True, 0, 0)
        ut2 = T.wino_weights(w, True, C, K)
        utb = T.wino_weights(w, True, C, K, True)
        R = max(T.wino_taylor_slots(S, S), 2)
        tay = torch.zeros(R, B, C, device=dev)
        bw = {
            "wino4": lambda: T.conv_wino4_dgrad(g, ut4, act, bn, tay, True, 0, 1, 0),
            "wino2": lambda: T.conv_wino_dgrad(g, None, ut2, act, bn, tay, True, 1, True),
            "wino2-bf16": lambda: T.conv_wino_dgrad(g, None, utb, act, bn, tay, True, 1, True),
        }
        row = {k: _time(f, args.iters) for k, f in bw.items()}
        for k, v in row.items():
            tot[("bwd", k)] = tot.get(("bwd", k), 0.0) + v
        print(f"{'':>22s} {'bwd':>5s} {row['wino4']:9.1f} {row['wino2']:9.1f} {row['wino2-bf16']:11.1f}", flush=True)
        del x, g, act
    for d in ("fwd", "bwd"):
        print(d, "totals:", {k: round(v, 1) for (dd, k), v in tot.items() if dd == d})


if __name__ == "__main__":
    main()
