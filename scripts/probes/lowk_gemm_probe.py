"""Memory-bound 1x1 convs of ResNet-50 training (short K, wide outputs: 64 -> 256 at 56 px,
B=128): every implicit-GEMM tile config with and without the BN-statistics epilogue, against
a plain device copy of the output size (the HBM reference). python scripts/probes/lowk_gemm_probe.py
[--one B S C N cfg stats]: a few launches of one shape / config (a PMC target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchpruner_amd import ops  # noqa: E402

T = ops.require()


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


if len(sys.argv) > 1 and sys.argv[1] == "--one":
    B, S, C, N, cfg, st = (int(v) for v in sys.argv[2:8])
    x = torch.randn(B, S, S, C, device="cuda")
    w = torch.randn(N, T.conv_gen_k(1, C), device="cuda") * 0.1
    for _ in range(5):
        if st:
            T.conv_gen_stats(x, w, None, 1, 1, 0, cfg)
        else:
            T.conv_gen(x, w, None, None, False, None, None, 1, 1, 0, cfg, 1)
    torch.cuda.synchronize()
    sys.exit(0)

for (B, S, C, N) in [(128, 56, 64, 256), (128, 56, 256, 64), (128, 56, 64, 64), (128, 28, 128, 512)]:
    x = torch.randn(B, S, S, C, device="cuda")
    w = torch.randn(N, T.conv_gen_k(1, C), device="cuda") * 0.1
    y = torch.empty(B, S, S, N, device="cuda")
    mb = (x.numel() + y.numel()) * 4 / 1e6
    y2 = torch.empty_like(y)
    cp = timeit(lambda: y2.copy_(y))
    rd = timeit(lambda: x.sum())
    print(f"B={B} S={S} {C}->{N}: in+out {mb:.0f} MB; copy(out) {cp:.1f} us, sum(in) {rd:.1f} us", flush=True)
    for cfg in list(range(7)) + [64 + 2, 64 + 3, 64 + 6]:  # 64 + c: single-buffered LDS stage (CFG_SB)
        try:
            t0 = timeit(lambda: T.conv_gen(x, w, None, None, False, None, None, 1, 1, 0, cfg, 1))
            t1 = timeit(lambda: T.conv_gen_stats(x, w, None, 1, 1, 0, cfg))
        except RuntimeError as e:
            print(f"  cfg {cfg}: {str(e)[:60]}")
            continue
        print(f"  cfg {cfg}: {t0:7.1f} us ({mb / t0:.2f} TB/s), with BN stats {t1:7.1f} us", flush=True)
