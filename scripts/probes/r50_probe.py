"""ResNet-50 B=64 eval forward on MIOpen (default vs deterministic) and the APoZ channel reduction
on a 64x64x112x112 NHWC activation: early-round timing references."""
import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import time, torch
import torch.nn.functional as F
from torchpruner_amd.models import resnet50
from torchpruner_amd import ops
m = resnet50().cuda().eval().to(memory_format=torch.channels_last)
x = torch.randn(64, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
def bench(name, fn, n=5):
    for i in range(2): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for i in range(n): fn()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / n
    print(f"{name}: {dt*1e3:.2f} ms", flush=True)
with torch.no_grad():
    bench("fwd default", lambda: m(x))
    torch.backends.cudnn.deterministic = True
    bench("fwd deterministic", lambda: m(x))
    torch.backends.cudnn.deterministic = False
    a = torch.relu(torch.randn(64, 64, 112, 112, device="cuda")).contiguous(memory_format=torch.channels_last)
    bench("apoz reduce NHWC 64x64x112x112", lambda: ops.channel_reduce(a, None, "apoz"))
    a2 = a.contiguous()
    bench("apoz reduce NCHW 64x64x112x112", lambda: ops.channel_reduce(a2, None, "apoz"))
m.train()
opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
y = torch.randint(0, 1000, (64,), device="cuda")
def step():
    opt.zero_grad(); F.cross_entropy(m(x), y).backward(); opt.step()
bench("train step default", step, 3)
torch.backends.cudnn.deterministic = True
bench("train step deterministic", step, 2)
