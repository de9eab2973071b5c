"""CPU check of the Winograd F(2x2,3x3) weight layout + transforms that winograd.hip assumes:
a PyTorch re-implementation of the kernel's algorithm (same B^T, A^T, interleaved U layout)
must reproduce F.conv2d."""
import torch
import torch.nn.functional as F

from torchpruner_amd.engine.fused_chain import winograd_weights

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def _decode_images(img):
    """(C/8, K/32, 4096) U images -> (4, 4, C, K)."""
    CB, KB = img.shape[0], img.shape[1]
    t = img.double().reshape(CB, KB, 16, 2, 16, 4, 2).clone()  # (cb, kb, xi, e, j, gs, n)
    t[:, :, :, :, 8:] = t[:, :, :, :, 8:, [2, 3, 0, 1]]
    t = t.permute(2, 0, 5, 3, 1, 6, 4)  # (xi, cb, g, e, kb, n, j)
    return t.reshape(4, 4, CB * 8, KB * 32)


def _wino_conv(x, u_img):
    """x (B,C,H,W) fp64; u_img = winograd_weights() images."""
    B, C, H, W = x.shape
    u = _decode_images(u_img)
    K = u.shape[3]
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
    assert u.shape == (1, 2, 4096)
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


def test_taylor_slots_cover_every_block():
    """Every 64-tile block touching an image maps to a distinct slot < taylor_slots(H, W)."""
    from torchpruner_amd.engine.fused_chain import taylor_slots
    for H, W in [(32, 32), (16, 16), (8, 8), (4, 4), (2, 2), (6, 10), (18, 14), (64, 32), (28, 28)]:
        T = (H // 2) * (W // 2)
        R = taylor_slots(H, W)
        for b in range(7):
            first = (b * T) // 64
            last = ((b + 1) * T - 1) // 64
            assert last - first + 1 <= R, (H, W, b)


def test_score_fold_slots_cpu_reference():
    import torch
    from torchpruner_amd import ops
    g = torch.Generator().manual_seed(0)
    T = torch.randn(3, 5, 4, generator=g)
    ref = T.sum(0).abs()
    acc = torch.zeros(4, dtype=torch.float64)
    ops.score_fold_([T], [acc], True, 1)
    torch.testing.assert_close(acc, ref.double().sum(0))
    torch.testing.assert_close(T[0], ref)
    assert torch.count_nonzero(T[1:]) == 0
