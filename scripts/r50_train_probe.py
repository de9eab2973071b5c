"""Probe: ResNet-50 fp32 SGD train-step time on one GPU, NCHW vs channels_last (MIOpen convs)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torchpruner_amd.models import resnet50  # noqa: E402

B = int(os.environ.get("B", 128))
fmts = os.environ.get("FMTS", "nchw,nhwc,native").split(",")
for fmt in fmts:
    torch.manual_seed(0)
    mf = torch.contiguous_format if fmt == "nchw" else torch.channels_last
    m = resnet50().cuda().to(memory_format=mf).train()
    if fmt == "native":
        from torchpruner_amd.engine.train import enable_native_convs
        print(f"native convs: {len(enable_native_convs(m))}", flush=True)
    fused = os.environ.get("OPT_FUSED", "0") != "0"  # torch's fused SGD (one kernel) vs foreach
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, **({"fused": True} if fused else {}))
    x = torch.randn(B, 3, 224, 224, device="cuda").contiguous(memory_format=mf)
    y = torch.randint(0, 1000, (B,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(m(x), y).backward()
        opt.step()

    t = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    print(f"{fmt} B={B}: warmup 3 steps {time.perf_counter() - t:.1f}s", flush=True)
    n = int(os.environ.get("N", 10))
    t = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / n
    print(f"{fmt} B={B}: {dt * 1e3:.1f} ms/step -> {B / dt:.0f} img/s", flush=True)
    del m, opt, x
    torch.cuda.empty_cache()
