"""F(4x4,3x3) (wino4.hip) vs the staged F(2x2,3x3) kernel (winograd.hip) on the VGG16-CIFAR
conv shapes at batch B: forward (BN+ReLU, pooled where VGG pools) and data gradient (W_BWD
epilogue with Taylor partials). Prints per-layer us and direct-conv-equivalent TFLOP/s.

    python scripts/wino4_bench.py [--batch 2048] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (S, Cin, Cout, pool) of VGG16 convs 2..13 (conv 1 has 3 input channels; 2x2 maps use the dense GEMM)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    B = args.batch
    tot = {"f2_fwd": 0.0, "f4_fwd": 0.0, "f2_bwd": 0.0, "f4_bwd": 0.0}
    print(f"B={B}: per layer us (direct-equivalent TF/s)")
    for S, C, K, pool in LAYERS:
        x = torch.randn(B, S, S, C, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) * 0.05
        sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
        u2 = T.wino_weights(w, False, 0, 0)
        u4 = T.wino4_weights(w, False, 0, 0)
        flop = 2.0 * B * S * S * C * K * 9
        t2 = timeit(lambda: T.conv_wino_fwd(x, u2, sc, sh, True, pool, 1, True, None), args.iters)
        t4 = timeit(lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None), args.iters)
        # dgrad of this layer: g (B,S,S,K) -> (B,S,S,C), act (B,S,S,C)
        g = torch.randn(B, S, S, K, device=dev)
        act = torch.relu(torch.randn(B, S, S, C, device=dev))
        scp = torch.rand(C, device=dev) + 0.5
        ut2 = T.wino_weights(w, True, 0, 0)
        ut4 = T.wino4_weights(w, True, 0, 0)
        R = max(T.wino_taylor_slots(S, S), 2)
        tay = torch.zeros(R, B, C, device=dev)
        b2 = b4 = float("nan")
        if C % 32 == 0:
            b2 = timeit(lambda: T.conv_wino_dgrad(g, None, ut2, act, scp, tay, True, 1, True, 0), args.iters)
            b4 = timeit(lambda: T.conv_wino4_dgrad(g, ut4, act, scp, tay, True, 0), args.iters)
        tot["f2_fwd"] += t2
        tot["f4_fwd"] += t4
        tot["f2_bwd"] += b2
        tot["f4_bwd"] += b4
        print(f"S={S:2d} C={C:3d} K={K:3d} pool={int(pool)} | fwd F2 {t2:7.1f} ({flop / t2 / 1e6:5.0f}) "
              f"F4 {t4:7.1f} ({flop / t4 / 1e6:5.0f}) x{t2 / t4:4.2f} | dgrad F2 {b2:7.1f} F4 {b4:7.1f} "
              f"x{b2 / b4:4.2f}", flush=True)
    print(f"total fwd F2 {tot['f2_fwd']:.0f} us F4 {tot['f4_fwd']:.0f} us (x{tot['f2_fwd'] / tot['f4_fwd']:.2f}); "
          f"dgrad F2 {tot['f2_bwd']:.0f} us F4 {tot['f4_bwd']:.0f} us (x{tot['f2_bwd'] / tot['f4_bwd']:.2f})")


if __name__ == "__main__":
    main()
