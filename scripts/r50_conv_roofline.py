"""Per-shape roofline of the ResNet-50 forward convolutions on the native kernels (B=256, fp32).

For every distinct conv shape of torchvision's ResNet-50 (stem, 1x1 / 3x3 / strided, downsample)
times every kernel candidate of the engine (implicit-GEMM tile configs x split-K, Winograd for
stride-1 3x3) with HIP events and reports the best, its direct-conv TFLOP/s, its HBM bytes
(input + weights + output; + the residual for the convs that carry the block's residual add in the
attribution engine) and the fraction of the roofline time max(FLOP / 155 TF, bytes / 5.5 TB/s).
Usage: python scripts/r50_conv_roofline.py [--batch 256] [--iters 10]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import TUNER, WINO, WINO_LDS, _wino_splits, cpad  # noqa: E402
from torchpruner_amd.models.resnet import resnet50  # noqa: E402

PEAK_TF, PEAK_TBS = 155.0, 5.5


def conv_shapes(batch):
    model = resnet50()
    shapes = collections.OrderedDict()
    hooks = []

    def hook(m, inp, out):
        x = inp[0]
        key = (m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0], m.padding[0], x.shape[2], x.shape[3])
        shapes[key] = shapes.get(key, 0) + 1

    for m in model.modules():
        if isinstance(m, torch.nn.Conv2d):
            hooks.append(m.register_forward_hook(hook))
    with torch.no_grad():
        model(torch.zeros(1, 3, 224, 224))
    for h in hooks:
        h.remove()
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ws", action="store_true", help="add the warp-specialised 1x1 GEMM cfgs (16-18)")
    ap.add_argument("--verbose", action="store_true", help="print every candidate's time")
    ap.add_argument("--hw", type=int, default=None, help="only the convs on this input size")
    args = ap.parse_args()
    T = ops.require()
    dev = torch.device("cuda")
    B = args.batch
    total_best = 0.0
    total_roof = 0.0
    print(f"{'cin':>5} {'cout':>5} {'k':>2} {'s':>2} {'hw':>4} {'n':>2} {'best':>24} {'us':>8} {'TF/s':>6} "
          f"{'TB/s':>6} {'roof%':>6}")
    for (cin, cout, ks, s, pad, H, W), n in conv_shapes(B).items():
        if args.hw is not None and H != args.hw:
            continue
        cin_p = 4 if (ks == 7 and cin <= 4) else cpad(cin)
        x = torch.randn(B, H, W, cin_p, device=dev)
        w = torch.randn(cout, cin_p, ks, ks, device=dev) * 0.05
        kk = T.conv_gen_k(ks, cin_p)
        wk = T.pack_conv_weight(w, cout, kk, cin_p, 0)
        Ho, Wo = (H + 2 * pad - ks) // s + 1, (W + 2 * pad - ks) // s + 1
        M = B * Ho * Wo
        scale = torch.ones(cout, device=dev)
        shift = torch.zeros(cout, device=dev)
        res = torch.randn(B, Ho, Wo, cout, device=dev) if (ks == 1 and cout >= 256 and s == 1 and cin < cout) else None
        cands = [(c, sp) for c, sp in TUNER.candidates(M, cout, kk)]
        if args.ws and ks == 1:
            cands += [(16, 1), (17, 1), (18, 1)]
        wino = ks == 3 and s == 1  # odd H / W: partial last tile row / column (as the engine)
        if wino:
            sp0 = _wino_splits(B * ((H + 1) // 2) * ((W + 1) // 2), cout, cin_p)
            u = T.wino_weights(w, False)
            cands = [(k, sp) for sp in sorted({1, 2, 4, sp0}) for k in (WINO_LDS, WINO)] + cands
        results = []
        for cfg, sp in cands:
            def run():
                if cfg in (WINO, WINO_LDS):
                    return T.conv_wino_fwd(x, u, scale, shift, True, False, sp, cfg == WINO_LDS)
                return T.conv_gen(x, wk, scale, shift, True, res, None, ks, s, pad, cfg, sp)
            try:
                run()
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            results.append((e0.elapsed_time(e1) / args.iters * 1e3, cfg, sp))
        us, cfg, sp = min(results)
        if args.verbose:
            print("   " + "  ".join(f"{c}/{p_}:{t:.0f}" for t, c, p_ in sorted(results, key=lambda r: (r[1], r[2]))))
        blas = ""
        if ks == 1 and s == 1:  # the same GEMM on hipBLASLt (torch.mm), no epilogue: a reference point
            a2, b2 = x.view(M, cin_p), w.view(cout, cin_p)
            torch.mm(a2, b2.t())
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                torch.mm(a2, b2.t())
            e1.record()
            torch.cuda.synchronize()
            blas = f"  hipBLASLt mm {e0.elapsed_time(e1) / args.iters * 1e3:.1f} us"
        flop = 2.0 * M * cout * cin * ks * ks
        byts = 4.0 * (B * H * W * cin_p + cout * kk + M * cout * (2 if res is not None else 1))
        roof = max(flop / (PEAK_TF * 1e12), byts / (PEAK_TBS * 1e12)) * 1e6
        total_best += us * n
        total_roof += roof * n
        name = {WINO: "wino", WINO_LDS: "wino_lds"}.get(cfg, f"igemm{cfg}") + f" sp{sp}"
        print(f"{cin:>5} {cout:>5} {ks:>2} {s:>2} {H:>4} {n:>2} {name:>24} {us:>8.1f} {flop / us / 1e6:>6.1f} "
              f"{byts / us / 1e6:>6.2f} {100 * roof / us:>5.0f}%{blas}", flush=True)
    print(f"sum over the network (x count): {total_best / 1e3:.2f} ms, roofline {total_roof / 1e3:.2f} ms "
          f"({100 * total_roof / total_best:.0f}%)")


if __name__ == "__main__":
    main()
