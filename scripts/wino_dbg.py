"""Time Winograd kernels with parts switched off (TP_WINO_DBG bits) on VGG16 layer shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.bench.conv_kernels import timeit  # noqa: E402
from torchpruner_amd.engine.fused_chain import taylor_slots, winograd_weights  # noqa: E402

T = ops.require()
dev = torch.device("cuda")
B = 512
for (H, W, C, K, pool) in [(32, 32, 64, 64, True), (8, 8, 256, 256, False), (4, 4, 512, 512, False)]:
    x = torch.randn(B, H, W, C, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.02
    u = winograd_weights(w)
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).contiguous())
    sc = torch.ones(K, device=dev)
    sh = torch.zeros(K, device=dev)
    act = torch.relu(torch.randn(B, H, W, C, device=dev))
    g = torch.randn(B, H, W, K, device=dev)
    tay = torch.zeros(taylor_slots(H, W), B, C, device=dev)
    scin = torch.ones(C, device=dev)
    for dbg in [int(v) for v in os.environ.get('DBGS', '0,1,2,4,3,7').split(',')]:
        os.environ["TP_WINO_DBG"] = str(dbg)
        tf = timeit(lambda: T.conv_wino_fwd(x, u, sc, sh, True, pool, 1, True), 10)
        tb = timeit(lambda: T.conv_wino_dgrad(g, None, ut, act, scin, tay, True, 1, True), 10)
        print(f"{H}x{W} {C}->{K} dbg={dbg}: fwd {tf:7.1f} us  dgrad {tb:7.1f} us", flush=True)
os.environ.pop("TP_WINO_DBG")
