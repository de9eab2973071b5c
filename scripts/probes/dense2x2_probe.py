"""The VGG16 2x2-map layers as dense GEMMs (engine/fused_chain.py DENSE: B x 4C -> 4N, here
2048 x 2048 x 2048 fp32): every implicit-GEMM tile config x split-K of the native kernel vs
hipBLASLt (torch.mm). python scripts/probes/dense2x2_probe.py [--m 2048] [--n 2048] [--k 2048]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import TUNER  # noqa: E402


def timeit(fn, iters=20):
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
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--k", type=int, default=2048)
    a = ap.parse_args()
    T = ops.require()
    dev = torch.device("cuda")
    x = torch.randn(a.m, 1, 1, a.k, device=dev)
    w = torch.randn(a.n, a.k, 1, 1, device=dev) * 0.02
    wk = T.pack_conv_weight(w, a.n, T.conv_gen_k(1, a.k), a.k, 0)
    sc, sh = torch.ones(a.n, device=dev), torch.zeros(a.n, device=dev)
    flop = 2.0 * a.m * a.n * a.k
    res = []
    for cfg, sp in TUNER.candidates(a.m, a.n, a.k) + [(c, s) for c in range(7) for s in (1, 2, 4)]:
        if any(r[1:] == (cfg, sp) for r in res):
            continue
        try:
            us = timeit(lambda: T.conv_gen(x, wk, sc, sh, True, None, None, 1, 1, 0, cfg, sp))
        except RuntimeError:
            continue
        res.append((us, cfg, sp))
    for us, cfg, sp in sorted(res):
        print(f"igemm cfg {cfg} sp {sp}: {us:8.1f} us {flop / us / 1e6:6.1f} TF/s", flush=True)
    a2, b2 = x.view(a.m, a.k), w.view(a.n, a.k)
    us = timeit(lambda: torch.mm(a2, b2.t()))
    print(f"hipBLASLt torch.mm (no epilogue): {us:8.1f} us {flop / us / 1e6:6.1f} TF/s")
    b3 = b2.t().contiguous()
    us = timeit(lambda: torch.mm(a2, b3))
    print(f"hipBLASLt torch.mm NN (no epilogue): {us:8.1f} us {flop / us / 1e6:6.1f} TF/s")


if __name__ == "__main__":
    main()
