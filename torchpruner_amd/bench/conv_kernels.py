"""Micro-benchmark of the fused conv kernels on the VGG16-CIFAR layer shapes (fwd + dgrad).

    python -m torchpruner_amd.bench.conv_kernels [--batch 256] [--iters 20] [--json out.json]

Reports time and TFLOP/s per layer (2*M*N*K / t) for the tile config the engine would pick,
and optionally every config (``--all-cfg``), so kernel changes can be A/B'd in one process.
"""
from __future__ import annotations

import argparse
import json

import torch

from torchpruner_amd import ops
from torchpruner_amd.engine.fused_chain import _pick_cfg, _wino_splits, winograd_weights

# (H, W, Cin, Cout, pool) of the 12 MFMA convs of VGG16 on 32x32 inputs
VGG16_LAYERS = [
    (32, 32, 64, 64, True),
    (16, 16, 64, 128, False),
    (16, 16, 128, 128, True),
    (8, 8, 128, 256, False),
    (8, 8, 256, 256, False),
    (8, 8, 256, 256, True),
    (4, 4, 256, 512, False),
    (4, 4, 512, 512, False),
    (4, 4, 512, 512, True),
    (2, 2, 512, 512, False),
    (2, 2, 512, 512, False),
    (2, 2, 512, 512, True),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--all-cfg", action="store_true")
    ap.add_argument("--wino", action="store_true", help="also time the Winograd kernel (splits sweep)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    T = ops.require()
    dev = torch.device("cuda")
    B = args.batch
    rows = []
    tot_f = tot_t = 0.0
    for li, (H, W, Cin, Cout, pool) in enumerate(VGG16_LAYERS):
        x = torch.randn(B, H, W, Cin, device=dev)
        w = torch.randn(Cout, 9 * Cin, device=dev) * 0.02
        wt = torch.randn(Cin, 9 * Cout, device=dev) * 0.02
        sc = torch.ones(Cout, device=dev)
        sh = torch.zeros(Cout, device=dev)
        M, flops = B * H * W, 2.0 * B * H * W * Cout * 9 * Cin
        act = torch.relu(torch.randn(B, H, W, Cin, device=dev))
        scin = torch.ones(Cin, device=dev)
        tay = torch.zeros(B, Cin, device=dev)
        if pool:
            g = torch.randn(B, H // 2, W // 2, Cout, device=dev)
            am = torch.randint(0, 4, (B, H // 2, W // 2, Cout), device=dev, dtype=torch.uint8)
        else:
            g = torch.randn(B, H, W, Cout, device=dev)
            am = None
        cfgs = [0, 1, 2, 3, 4, 5, 6] if args.all_cfg else [None]
        for cfg in cfgs:
            fc, fs = _pick_cfg(M, Cout, 9 * Cin)
            bc, bs = _pick_cfg(M, Cin, 9 * Cout)
            if cfg is not None:
                fc = bc = cfg
            tf = timeit(lambda: T.conv_fwd(x, w, sc, sh, True, pool, 3, fc, fs), args.iters)
            tb = timeit(lambda: T.conv_dgrad(g, am, wt, act, scin, tay, True, 3, bc, bs), args.iters)
            r = {"layer": li + 1, "shape": [B, H, W, Cin, Cout], "pool": pool, "fwd_cfg": [fc, fs], "bwd_cfg": [bc, bs],
                 "fwd_us": round(tf, 1), "bwd_us": round(tb, 1), "fwd_tflops": round(flops / tf / 1e6, 1),
                 "bwd_tflops": round(flops / tb / 1e6, 1)}
            rows.append(r)
            if cfg is None:
                tot_f += 2 * flops
                tot_t += tf + tb
            print(f"L{li+1:2d} {H:2d}x{W:<2d} {Cin:3d}->{Cout:3d} pool={int(pool)} cfg f{fc}/{fs} b{bc}/{bs}: "
                  f"fwd {tf:7.1f} us {flops/tf/1e6:6.1f} TF | dgrad {tb:7.1f} us {flops/tb/1e6:6.1f} TF", flush=True)
        if args.wino:
            # TF/s columns are direct-conv-equivalent FLOPs (2*M*N*9*C) / time
            u = winograd_weights(w.view(Cout, 3, 3, Cin).permute(0, 3, 1, 2))
            ut = winograd_weights(wt.view(Cin, 3, 3, Cout).permute(0, 3, 1, 2))
            P = B * (H // 2) * (W // 2)
            base_f, base_b = _wino_splits(P, Cout, Cin), _wino_splits(P, Cin, Cout)
            for staged in (False, True):
                for sf, sb in sorted({(base_f, base_b), (1, 1), (max(1, base_f // 2), max(1, base_b // 2)),
                                      (base_f * 2, base_b * 2)}):
                    tf = timeit(lambda: T.conv_wino_fwd(x, u, sc, sh, True, pool, sf, staged), args.iters)
                    tb = timeit(lambda: T.conv_wino_dgrad(g, am, ut, act, scin, tay, True, sb, staged), args.iters)
                    rows.append({"layer": li + 1, "wino": "lds" if staged else "direct", "splits": [sf, sb],
                                 "fwd_us": round(tf, 1), "bwd_us": round(tb, 1)})
                    print(f"    wino-{'lds' if staged else 'dir'} splits f{sf}/b{sb}: fwd {tf:7.1f} us "
                          f"{flops/tf/1e6:6.1f} TFe | dgrad {tb:7.1f} us {flops/tb/1e6:6.1f} TFe", flush=True)
    if tot_t:
        print(f"TOTAL {tot_t:.1f} us, {tot_f / tot_t / 1e6:.1f} TF/s average")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"batch": B, "rows": rows, "total_us": tot_t}, f, indent=1)


if __name__ == "__main__":
    main()
