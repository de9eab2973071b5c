"""The opt-in bf16 Taylor engine on the headline shape (VGG16-BN/CIFAR, B=2048, random init):
a few tuned steps, for a kernel-trace breakdown of one bf16 step (scripts/step_breakdown.py).
python scripts/probes/bf16_step_probe.py [--steps 4] [--fp32]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--fp32", action="store_true")
    args = ap.parse_args()
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import vgg_cifar
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = vgg_cifar(16).to(dev).eval()
    convs = [m for m in model.modules() if isinstance(m, torch.nn.Conv2d)]
    B = args.batch
    x = torch.randn(B, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    kw = {} if args.fp32 else {"compute_dtype": torch.bfloat16}
    run = lambda: TaylorAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, dev,  # noqa: E731
                                          **kw).run_many(convs, find_best_evaluation_module=True)
    run()  # tune
    torch.cuda.synchronize()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
