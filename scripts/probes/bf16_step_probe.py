"""The opt-in bf16 VGG16 Taylor engine step at B=2048 (random-init weights, synthetic batches): a
few tuned warm-up batches, then --steps timed batches; a target for rocprofv3 --kernel-trace
--stats (the step's per-kernel breakdown). python scripts/probes/bf16_step_probe.py [--steps 5] [--fp32]"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--pin", default=None, help="kernel family pinned for every layer it covers (fused_chain.family_policy)")
    args = ap.parse_args()
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine.fused_chain import TUNER, family_policy
    from torchpruner_amd.models import prunable_vgg16
    import contextlib
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    dt = None if args.fp32 else torch.bfloat16
    B = args.batch
    x = torch.randn(B * args.steps, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (B * args.steps,), device=dev)
    ctx = TUNER.pinned(family_policy(args.pin)) if args.pin else contextlib.nullcontext()
    with ctx:
        TaylorAttributionMetric(model, DeviceLoader(x[:2 * B], y[:2 * B], B), F.cross_entropy, dev,
                                compute_dtype=dt).run_many(convs, True)  # tune
        torch.cuda.synchronize()
        m = TaylorAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, dev, compute_dtype=dt)
        t0 = time.perf_counter()
        m.run_many(convs, True)
        torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
        if os.environ.get("PROBE_CHOICES"):
            for k, v in TUNER.cache.items():
                print("  choice", k, "->", v)
    print(f"{'fp32' if args.fp32 else 'bf16'} pin={args.pin} B={B}: {dt_s / args.steps * 1e3:.2f} ms/step, "
          f"{B * args.steps / dt_s:.0f} img/s, path {m.last_path['path']}", flush=True)


if __name__ == "__main__":
    main()
