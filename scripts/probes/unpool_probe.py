"""Bandwidth of the argmax unpooling kernel (prune_ops.hip unpool2_nhwc_v4) at the VGG16/CIFAR
pooled-layer shapes, B=2048 fp32: us per launch and GB/s (gradient + argmax read, full-size
gradient written). python scripts/probes/unpool_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import ops  # noqa: E402


def main():
    T = ops.require()
    dev = torch.device("cuda")
    B = 2048
    for H, C in ((32, 64), (16, 128), (8, 256), (4, 512)):
        x = torch.randn(B, H, H, C, device=dev)
        y, am = T.maxpool2_nhwc(x)
        g = torch.randn_like(y)
        T.unpool2_nhwc(g, am)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            T.unpool2_nhwc(g, am)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        byts = g.numel() * 4 + am.numel() * am.element_size() + x.numel() * 4
        print(f"H={H:>2} C={C:>3}: {us:7.1f} us {byts / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
