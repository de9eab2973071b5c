"""Does the Winograd kernel's speed depend on the operand VALUES (MFMA power / clock behaviour)?

Times the staged forward kernel (no epilogue work beyond the store) on one VGG16 layer shape with
the same launch geometry and three inputs: dense N(0,1), ReLU'd N(0,1) (~50% zeros, like the
forward's post-ReLU activations) and all zeros; and the dgrad kernel with dense vs sparse gradients.
Usage: python scripts/probes/wino_data_dependence.py [--batch 2048]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import winograd_weights  # noqa: E402


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    T = ops.require()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for (H, C, K) in ((8, 256, 256), (16, 128, 128), (32, 64, 64)):
        B = args.batch
        w = torch.randn(K, C, 3, 3, device=dev) * (2.0 / (9 * C)) ** 0.5
        u = winograd_weights(w)
        ut = winograd_weights(w.flip(2, 3).transpose(0, 1).contiguous())
        dense = torch.randn(B, H, H, C, device=dev)
        inputs = {"dense": dense, "relu": torch.relu(dense), "zeros": torch.zeros_like(dense)}
        res = {k: bench(lambda x=x: T.conv_wino_fwd(x, u, None, None, False, False, 1, True)) for k, x in inputs.items()}
        act = torch.relu(torch.randn(B, H, H, C, device=dev))
        gd = torch.randn(B, H, H, K, device=dev)
        gin = {"dense": gd, "relu": torch.relu(gd), "zeros": torch.zeros_like(gd)}
        resb = {k: bench(lambda g=g: T.conv_wino_dgrad(g, None, ut, act, None, None, True, 1, True, 0))
                for k, g in gin.items()}
        print(f"H={H} C={C} K={K} B={B}: fwd " + " ".join(f"{k} {v:.1f}us" for k, v in res.items())
              + " | dgrad " + " ".join(f"{k} {v:.1f}us" for k, v in resb.items()), flush=True)


if __name__ == "__main__":
    main()
