"""A few launches of Winograd fwd vs unpool-dgrad on VGG16 layer shapes, for PMC runs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import taylor_slots, winograd_weights  # noqa: E402

T = ops.require()
dev = torch.device("cuda")
B = 512
for (H, W, C, K) in [(32, 32, 64, 64), (16, 16, 128, 128)]:
    x = torch.randn(B, H, W, C, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.02
    u = winograd_weights(w)
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).contiguous())
    sc = torch.ones(K, device=dev)
    sh = torch.zeros(K, device=dev)
    gp = torch.randn(B, H // 2, W // 2, K, device=dev)
    am = torch.randint(0, 4, (B, H // 2, W // 2, K), device=dev, dtype=torch.uint8)
    act = torch.relu(torch.randn(B, H, W, C, device=dev))
    tay = torch.zeros(taylor_slots(H, W), B, C, device=dev)
    scin = torch.ones(C, device=dev)
    for _ in range(3):
        T.conv_wino_fwd(x, u, sc, sh, True, True, 1, True)
    for _ in range(3):
        T.conv_wino_dgrad(gp, am, ut, act, scin, tay, False, 1, True)
    for _ in range(3):
        T.conv_wino_dgrad(gp, am, ut, act, scin, None, False, 1, True)
    gfull = torch.randn(B, H, W, K, device=dev)
    for _ in range(3):
        T.conv_wino_dgrad(gfull, None, ut, act, scin, tay, False, 1, True)
torch.cuda.synchronize()
print("ok")
