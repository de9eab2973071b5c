"""CPU check of the Winograd F(2x2,3x3) weight layout + transforms that winograd.hip assumes:
a PyTorch re-implementation of the kernel's algorithm (same B^T, A^T, interleaved U layout)
must reproduce F.conv2d."""
import torch
import torch.nn.functional as F

from torchpruner_amd.engine.fused_chain import winograd_weights

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def _wino_conv(x, u_il):
    """x (B,C,H,W) fp64; u_il (16, C, K) in the kernel's interleaved layout."""
    B, C, H, W = x.shape
    K = u_il.shape[2]
    u = u_il.double().reshape(16, C, K // 32, 16, 2).transpose(3, 4).reshape(4, 4, C, K)
    xp = F.pad(x, (1, 1, 1, 1))
    patches = xp.unfold(2, 4, 2).unfold(3, 4, 2)  # (B, C, H/2, W/2, 4, 4)
    V = torch.einsum("ir,bcpqrs,js->bpqijc", BT, patches, BT)
    M = torch.einsum("bpqijc,ijck->bpqijk", V, u)
    Y = torch.einsum("ai,bpqijk,cj->bkpaqc", AT, M, AT)  # (B, K, H/2, 2, W/2, 2)
    return Y.reshape(B, K, H, W)


def test_winograd_layout_matches_conv2d():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 8, 6, 10, generator=g, dtype=torch.float64)
    w = torch.randn(64, 8, 3, 3, generator=g, dtype=torch.float64)
    u = winograd_weights(w.float())
    assert u.shape == (16, 8, 64)
    ref = F.conv2d(x, w, padding=1)
    got = _wino_conv(x, u)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_winograd_dgrad_weights():
    g = torch.Generator().manual_seed(1)
    w = torch.randn(32, 64, 3, 3, generator=g, dtype=torch.float64)  # conv 64 -> 32
    gy = torch.randn(2, 32, 4, 6, generator=g, dtype=torch.float64)
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).float())  # (16, 32, 64)
    ref = torch.nn.grad.conv2d_input((2, 64, 4, 6), w, gy, padding=1)
    torch.testing.assert_close(_wino_conv(gy, ut), ref, rtol=1e-5, atol=1e-5)
