"""One Winograd layer (default S=8, C=K=256, B=2048, forward) launched a few times: a target for
rocprofv3 PMC passes. --kind wino4 (F(4x4) fp32), wino2 (F(2x2) staged fp32) or wino2bf (F(2x2)
staged, bf16 U images + bf16 MFMA).
python scripts/probes/wino4_layer_probe.py [--S 8 --C 256 --K 256 --variant 0 --kind wino4]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=8)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--kind", default="wino4", choices=["wino4", "wino2", "wino2bf"])
    ap.add_argument("--dgrad", action="store_true", help="the data gradient (Taylor epilogue) instead of the forward")
    ap.add_argument("--pool", action="store_true")
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    S, C, K, B = args.S, args.C, args.K, args.B
    x = torch.randn(B, S, S, C, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.05
    sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    if args.dgrad:  # x plays the K-channel output gradient: dgrad of a conv C -> K is K -> C
        g = torch.randn(B, S, S, K, device=dev)
        act = torch.relu(torch.randn(B, S, S, C, device=dev))
        tay = torch.zeros(max(T.wino_taylor_slots(S, S), 2), B, C, device=dev)
        if args.kind == "wino4":
            ut = T.wino4_weights(w, True, 0, 0)
            run = lambda: T.conv_wino4_dgrad(g, ut, act, sc[:C] if C <= K else None, tay, True, 0, 1, args.variant)  # noqa: E731
        else:
            ut = T.wino_weights(w, True, C, K, args.kind == "wino2bf")
            run = lambda: T.conv_wino_dgrad(g, None, ut, act, None, tay, True, 1, True)  # noqa: E731
    elif args.kind == "wino4":
        u4 = T.wino4_weights(w, False, 0, 0)
        run = lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, args.pool, None, 1, args.variant)  # noqa: E731
    else:
        u2 = T.wino_weights(w, False, K, C, args.kind == "wino2bf")
        run = lambda: T.conv_wino_fwd(x, u2, sc, sh, True, args.pool, 1, True)  # noqa: E731
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
