"""A/B the conv_gen forward epilogue (TP_GEN_EPI) on the ResNet-50 engine, same process."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchpruner_amd.engine.resnet_engine import ResNetEngine, build_resnet_plan  # noqa: E402
from torchpruner_amd.models import resnet50  # noqa: E402

dev = torch.device("cuda")
model = resnet50().to(dev).eval()
eng = ResNetEngine(model, build_resnet_plan(model)[0])
x = torch.randn(256, 3, 224, 224, device=dev)
with torch.no_grad():
    for mode in ("1", "0", "1", "0"):
        os.environ["TP_GEN_EPI"] = mode
        eng.forward(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            eng.forward(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(f"TP_GEN_EPI={mode}: {dt*1e3:.2f} ms/batch -> {256/dt:.0f} img/s", flush=True)
