"""Stream-K vs data-parallel launches of the native 1x1 / 3x3 implicit GEMM on the ResNet-50 B=256
conv shapes (forward, BN-free; and the stride-1 1x1 data gradients), against hipBLASLt fp32
(torch.mm on the pre-gathered (M, K) operand: no im2col / stride gather counted). Per shape: the
best data-parallel (cfg, splits) of the tuner's candidate list (+ the persistent 1x1 cfgs 16-18),
the best stream-K cfg, and TF/s of each.
python scripts/probes/streamk_probe.py [--B 256] [--dgrad]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

# (Cin, Cout, H_in, ks, stride): the distinct ResNet-50 (torchvision v1.5) forward convs
SHAPES = [(64, 64, 56, 1, 1), (64, 256, 56, 1, 1), (256, 64, 56, 1, 1), (256, 128, 56, 1, 1), (256, 512, 56, 1, 2),
          (128, 512, 28, 1, 1), (512, 128, 28, 1, 1), (512, 256, 28, 1, 1), (512, 1024, 28, 1, 2),
          (256, 1024, 14, 1, 1), (1024, 256, 14, 1, 1), (1024, 512, 14, 1, 1), (1024, 2048, 14, 1, 2),
          (512, 2048, 7, 1, 1), (2048, 512, 7, 1, 1),
          (64, 64, 56, 3, 1), (128, 128, 28, 3, 1), (256, 256, 14, 3, 1), (512, 512, 7, 3, 1)]


def timeit(fn, iters=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(rounds):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--dgrad", action="store_true")
    args = ap.parse_args()
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import CFG_SK, TUNER, kernel_name, sk_candidates
    T = ops.require()
    dev = torch.device("cuda")
    B = args.B
    tot = {"dp": 0.0, "sk": 0.0, "blas": 0.0}
    for cin, cout, hw, ks, s in SHAPES:
        if args.dgrad and (ks != 1 or s != 1):
            continue
        pad = ks // 2
        ho = (hw + 2 * pad - ks) // s + 1
        M = B * ho * ho
        if args.dgrad:  # dgrad of cin -> cout: a (M, cout) x (cout, cin) GEMM with the ReLU mask
            g = torch.randn(B, hw, hw, cout, device=dev)
            wt = torch.randn(cin, cout, device=dev) * cout ** -0.5
            mask = torch.relu(torch.randn(B, hw, hw, cin, device=dev))
            N, K = cin, cout
            run = lambda c, sp: T.conv_gen_bwd(g, wt, None, 1, mask, 1, 1, 0, hw, hw, False, c, sp, None, 0)  # noqa
            a2, b2 = g.reshape(M, K), wt.t().contiguous()
        else:
            x = torch.randn(B, hw, hw, cin, device=dev)
            kk = T.conv_gen_k(ks, cin)
            w = torch.randn(cout, cin, ks, ks, device=dev) * 0.02
            wk = T.pack_conv_weight(w, cout, kk, cin, 0)
            N, K = cout, kk
            run = lambda c, sp: T.conv_gen(x, wk, None, None, False, None, None, ks, s, pad, c, sp)  # noqa
            a2 = torch.randn(M, K, device=dev)
            b2 = torch.randn(K, N, device=dev)
        cands = TUNER.candidates(M, N, K)
        if ks == 1:
            cands = cands + [(c, 1) for c in (16, 17, 18)]
        dp = min((timeit(lambda: run(c, sp)), c, sp) for c, sp in cands)
        skc = sk_candidates(T, cands, ks, M, N)
        sk = min(((timeit(lambda: run(c, 1)), c, 1) for c, _ in skc), default=(float("inf"), -1, 1))
        blas = timeit(lambda: torch.mm(a2, b2))
        fl = 2.0 * M * N * K
        best = min(dp[0], sk[0])
        tot["dp"] += dp[0]
        tot["sk"] += best
        tot["blas"] += blas
        print(f"{'dgrad' if args.dgrad else 'fwd'} {cin:5d}->{cout:5d} k{ks} s{s} @{hw:2d} M={M:6d}: "
              f"dp {dp[0]:7.1f}us {fl / dp[0] / 1e6:6.1f}TF ({kernel_name(dp[1])},{dp[2]})  "
              f"sk {sk[0]:7.1f}us {fl / sk[0] / 1e6 if sk[1] >= 0 else 0:6.1f}TF "
              f"({kernel_name(sk[1]) if sk[1] >= 0 else '-'})  hipblaslt {blas:7.1f}us {fl / blas / 1e6:6.1f}TF  "
              f"best/blas {best / blas:5.2f}", flush=True)
    print(f"sum: dp {tot['dp']:.0f}us  best(dp,sk) {tot['sk']:.0f}us  hipblaslt {tot['blas']:.0f}us", flush=True)
    assert CFG_SK == 32


if __name__ == "__main__":
    main()
