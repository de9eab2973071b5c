"""Diagnose the bf16 F(2x2) kernel against its emulation (tests/test_wino_bf16_gpu.py): error
norm, fraction of bad elements, and where they sit (per tile position / channel block / chunk)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import test_wino_bf16_gpu as t  # noqa: E402


def main():
    from torchpruner_amd import ops
    T = ops.require()
    dev = torch.device("cuda")
    for (B, H, W, C, K) in [(4, 32, 32, 64, 64), (3, 16, 16, 128, 256), (5, 8, 8, 256, 256), (6, 4, 4, 512, 512)]:
        g = torch.Generator().manual_seed(3 + H * C)
        x = torch.randn(B, H, W, C, generator=g)
        w = torch.randn(K, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5
        ub = T.wino_weights(w.to(dev), False, K, C, True)
        out, _ = T.conv_wino_fwd(x.to(dev), ub, None, None, False, False, 1, True)
        emu = t._wino_bf16_conv(x, w)
        d = (out.cpu().double() - emu).abs()
        bad = d > 1e-3 * emu.abs().max()
        print((B, H, W, C, K), "rel", float((out.cpu().double() - emu).norm() / emu.norm()),
              "bad frac", float(bad.float().mean()), flush=True)
        if bad.any():
            idx = bad.nonzero()
            print("  bad per image", torch.bincount(idx[:, 0], minlength=B).tolist())
            print("  bad per row%4", torch.bincount(idx[:, 1] % 4, minlength=4).tolist(),
                  "per col%4", torch.bincount(idx[:, 2] % 4, minlength=4).tolist())
            print("  bad per k%32", torch.bincount(idx[:, 3] % 32, minlength=32).tolist())
            print("  bad per k//32", torch.bincount(idx[:, 3] // 32).tolist())


if __name__ == "__main__":
    main()
