"""A few launches of the Winograd and direct kernels on two VGG16 layer shapes, for PMC runs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchpruner_amd import ops  # noqa: E402
from torchpruner_amd.engine.fused_chain import winograd_weights  # noqa: E402

T = ops.require()
dev = torch.device("cuda")
B = 512
for (H, W, C, K, pool) in [(32, 32, 64, 64, True), (4, 4, 512, 512, False)]:
    x = torch.randn(B, H, W, C, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.02
    u = winograd_weights(w)
    wk = w.permute(0, 2, 3, 1).reshape(K, -1).contiguous()
    sc = torch.ones(K, device=dev)
    sh = torch.zeros(K, device=dev)
    for _ in range(3):
        T.conv_wino_fwd(x, u, sc, sh, True, pool, 1)
    for _ in range(3):
        T.conv_fwd(x, wk, sc, sh, True, pool, 3, 3, 1)
torch.cuda.synchronize()
print("ok")
