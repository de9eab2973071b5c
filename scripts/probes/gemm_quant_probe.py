"""Does tile quantisation (work rounds over the 256-CU grid) bound the ResNet-50 1x1 GEMMs? Times
the native 1x1 conv (conv_gen, fwd, BN-free) at B=256 (M = 50176 / 12544 / 200704: 392 / 98 /
1568 tiles of 128 rows, i.e. x.06 rounds of 512 block slots) and at batch sizes that make the tile
count a whole number of rounds, per tile config; TF/s per point."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    for cin, cout, hw in ((1024, 256, 14), (256, 1024, 14), (2048, 512, 7), (512, 128, 28)):
        w = torch.randn(cout, cin, 1, 1, device=dev) * 0.02
        kk = T.conv_gen_k(1, cin)
        wk = T.pack_conv_weight(w, cout, kk, cin, 0)
        for B in (256, 320, 334, 384):
            x = torch.randn(B, hw, hw, cin, device=dev)
            M = B * hw * hw
            row = f"{cin:5d}->{cout:5d} @{hw:2d} B={B:3d} M={M:6d}:"
            for cfg in (4, 2, 6):
                t = timeit(lambda: T.conv_gen(x, wk, None, None, False, None, None, 1, 1, 0, cfg, 1))
                row += f"  cfg{cfg} {t:7.1f}us {2 * M * cout * cin / t / 1e6:6.1f}TF"
            print(row, flush=True)


if __name__ == "__main__":
    main()
