"""Probe: hipBLASLt (torch.mm, fp32) on the headline's dense 2x2-layer GEMMs (VGG16 layers 34/37/40
as B x 4C by 4C x 4K GEMMs at B=2048: 2048^3) next to the engine's own tile choices for the same
shapes (bench tuner log: dense2x2_igemm128x128, 2 splits, ~148-171 us per launch).

    python scripts/probes/dense_blas_probe.py
"""
import torch


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    dev = torch.device("cuda")
    torch.backends.cuda.matmul.allow_tf32 = False
    for (m, k, n) in [(2048, 2048, 2048), (2048, 2048, 512), (2048, 512, 2048)]:
        a = torch.randn(m, k, device=dev)
        b = torch.randn(k, n, device=dev)
        bt = b.t().contiguous()
        us = bench(lambda: torch.mm(a, b))
        us_t = bench(lambda: torch.mm(a, bt.t()))
        tf = 2 * m * n * k / us * 1e-6
        print(f"[dense_blas] {m}x{k}x{n}: torch.mm {us:.1f} us ({tf:.1f} TF/s), B^T layout {us_t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
