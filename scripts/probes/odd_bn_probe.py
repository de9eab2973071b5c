"""Training BatchNorm + ReLU on channel counts the native kernels do not take (C % 4 != 0, e.g.
103 / 205 / 410 after config #5's 20% prune): the library path (nn.BatchNorm2d on a channels_last
tensor, then ReLU) vs the native kernels on a 4-padded copy (pad, native BN+ReLU, slice back),
forward + backward, B=128. python scripts/probes/odd_bn_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torchpruner_amd.engine import train as tr  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for (C, S) in [(103, 28), (205, 14), (410, 7), (52, 56), (42, 56)]:
    x = torch.randn(128, C, S, S, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_()
    bn = torch.nn.BatchNorm2d(C).cuda().train()
    g = torch.randn_like(x)

    def lib():
        y = F.relu(bn(x))
        y.backward(g)

    Cp = -(-C // 4) * 4
    bnp = torch.nn.BatchNorm2d(Cp).cuda().train()

    def padded():
        xp = F.pad(x, (0, 0, 0, 0, 0, Cp - C)).contiguous(memory_format=torch.channels_last)
        y = tr.bn_act(bnp, xp, relu=True)[:, :C]
        y.backward(g)

    t_lib = timeit(lib)
    t_pad = timeit(padded) if C % 4 else float("nan")
    t_nat = timeit(lambda: tr.bn_act(bn, x, relu=True).backward(g)) if C % 4 == 0 else float("nan")
    print(f"C={C} S={S}: library {t_lib:.1f} us, native on 4-padded copy {t_pad:.1f} us, native direct {t_nat:.1f} us",
          flush=True)
