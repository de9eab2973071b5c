"""Kernel under PMC: the 1x1 implicit-GEMM conv (fwd, BN+ReLU epilogue) on two compute-bound
ResNet-50 shapes at B=256 with fixed tile configs, 10 launches each (rocprofv3 --pmc target)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchpruner_amd import ops  # noqa: E402


def main():
    T = ops.require()
    dev = torch.device("cuda")
    for (cin, cout, hw, cfg) in ((512, 128, 28, 4), (1024, 256, 14, 2), (256, 1024, 14, 4)):
        x = torch.randn(256, hw, hw, cin, device=dev)
        w = torch.randn(cout, cin, device=dev) * 0.05
        sc, sh = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
        for _ in range(10):
            T.conv_gen(x, w, sc, sh, True, None, None, 1, 1, 0, cfg, 1)
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
