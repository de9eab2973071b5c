"""One F(4x4) layer (default S=8, C=K=256, B=2048, forward) launched a few times: a target for
rocprofv3 PMC passes. python scripts/wino4_layer_probe.py [--S 8 --C 256 --K 256 --variant 0 --dgrad]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=8)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    S, C, K, B = args.S, args.C, args.K, args.B
    x = torch.randn(B, S, S, C, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.05
    sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    u4 = T.wino4_weights(w, False, 0, 0)
    for _ in range(args.iters):
        T.conv_wino4_fwd(x, u4, sc, sh, True, False, None, 1, args.variant)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
