"""Probe: Winograd F(4x4,3x3) forward (csrc/probe/wino_f4x3.hip) vs the engine's F(2x2,3x3)
kernels on the VGG16-CIFAR layer shapes: max error vs an fp64 reference, time, TFLOP/s
(direct-conv equivalent).   python csrc/probe/wino4_probe.py [B]"""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.bench.conv_kernels import timeit  # noqa: E402
from torchpruner_amd.engine.fused_chain import _wino_splits, winograd_weights  # noqa: E402

G4 = [[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
      [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]]


def u4(w):
    K, C = w.shape[:2]
    G = torch.tensor(G4, dtype=torch.float64, device=w.device)
    u = torch.einsum("ia,kcab,jb->ijck", G, w.double(), G).reshape(36, C // 4, 4, K // 16, 16)
    return u.permute(1, 3, 0, 2, 4).contiguous().float()


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = ctypes.CDLL(os.path.join(HERE, "wino4.so"))
    T = ops.require()
    dev = torch.device("cuda")
    P = ctypes.c_void_p
    for H, C, K in [(32, 64, 64), (16, 64, 128), (16, 128, 128), (8, 128, 256), (8, 256, 256), (4, 256, 512),
                    (4, 512, 512)]:
        torch.manual_seed(H * 1000 + C)
        x = torch.randn(B, H, H, C, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) * (2.0 / (9 * C)) ** 0.5
        sc = torch.rand(K, device=dev) + 0.5
        sh = torch.randn(K, device=dev) * 0.1
        out = torch.empty(B, H, H, K, device=dev)
        U4 = u4(w)
        st = torch.cuda.current_stream().cuda_stream

        def run4():
            rc = lib.tp_probe_wino4_fwd(P(x.data_ptr()), P(U4.data_ptr()), P(sc.data_ptr()), P(sh.data_ptr()),
                                        P(out.data_ptr()), B, H, H, C, K, 1, P(st))
            assert rc == 0, rc

        run4()
        torch.cuda.synchronize()
        nb = 32
        ref = torch.relu(F.conv2d(x[:nb].permute(0, 3, 1, 2).double(), w.double(), padding=1) *
                         sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)).permute(0, 2, 3, 1)
        err4 = ((out[:nb].double() - ref).abs().max() / ref.abs().max()).item()
        U2 = winograd_weights(w)
        sp = _wino_splits(B * (H // 2) * (H // 2), K, C)
        o2, _ = T.conv_wino_fwd(x, U2, sc, sh, True, False, sp, True)
        err2 = ((o2[:nb].double() - ref).abs().max() / ref.abs().max()).item()
        flops = 2.0 * B * H * H * K * 9 * C
        t4 = timeit(run4, 20)
        res = []
        for staged in (False, True):
            for s_ in sorted({sp, max(1, sp // 2), 1}):
                t = timeit(lambda s_=s_, st_=staged: T.conv_wino_fwd(x, U2, sc, sh, True, False, s_, st_), 20)
                res.append((t, staged, s_))
        t2, stg, s2 = min(res)
        print(f"H={H:2d} C={C:3d} K={K:3d}: F4 {t4:8.1f} us {flops / t4 / 1e6:6.1f} TF err {err4:.1e} | "
              f"F2 best {t2:8.1f} us {flops / t2 / 1e6:6.1f} TF (staged={stg}, splits={s2}) err {err2:.1e} | "
              f"speedup {t2 / t4:.2f}x", flush=True)


if __name__ == "__main__":
    main()
