"""A few launches of the F(4x4) and F(2x2) forward kernels on one VGG16 layer shape, for PMC runs:
``python scripts/probes/wino4_probe.py S C K [B]``."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchpruner_amd import ops  # noqa: E402

T = ops.require()
dev = torch.device("cuda")
S, C, K = (int(v) for v in sys.argv[1:4])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 2048
x = torch.randn(B, S, S, C, device=dev)
w = torch.randn(K, C, 3, 3, device=dev) * 0.05
sc, sh = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
u2, u4 = T.wino_weights(w, False, 0, 0), T.wino4_weights(w, False, 0, 0)
for _ in range(3):
    T.conv_wino4_fwd(x, u4, sc, sh, True, False, None)
    T.conv_wino_fwd(x, u2, sc, sh, True, False, 1, True, None)
torch.cuda.synchronize()
print("probe ok")
