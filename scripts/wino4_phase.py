"""Phase costs of the F(4x4) kernels: per-layer us at B for the current TP_W4_DBG setting (1 no U
DMA, 2 no X DMA, 16 no epilogue; results are WRONG when set — timing only). Run once per setting:

    for d in 0 1 2 3 16 19; do TP_W4_DBG=$d python scripts/wino4_phase.py --variant 0; done
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

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
    ap.add_argument("--variant", type=int, default=0)
    args = ap.parse_args()
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    B = args.batch
    row = []
    for S, C, K, pool in LAYERS:
        x = torch.randn(B, S, S, C, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) * 0.05
        sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
        u4 = T.wino4_weights(w, False, 0, 0)
        tf = timeit(lambda: T.conv_wino4_fwd(x, u4, sc, sh, True, pool, None, 1, args.variant), args.iters)
        g = torch.randn(B, S, S, K, device=dev)
        act = torch.relu(torch.randn(B, S, S, C, device=dev))
        ut4 = T.wino4_weights(w, True, 0, 0)
        tay = torch.zeros(4, B, C, device=dev)
        scp = torch.rand(C, device=dev) + 0.5
        tb = timeit(lambda: T.conv_wino4_dgrad(g, ut4, act, scp, tay, True, 0, 1, args.variant),
                    args.iters) if C % 32 == 0 else 0.0
        row.append((tf, tb))
    d = os.environ.get("TP_W4_DBG", "0")
    print(f"dbg={d:>2} variant={args.variant} B={B} fwd/dgrad us: " +
          " ".join(f"{f:.0f}/{b:.0f}" for f, b in row) + f" | total {sum(f for f, _ in row):.0f}/"
          f"{sum(b for _, b in row):.0f}", flush=True)


if __name__ == "__main__":
    main()
