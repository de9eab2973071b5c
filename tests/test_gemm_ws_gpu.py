"""Persistent warp-specialised 1x1 GEMM (gemm_ws.hip, conv_gen cfgs 16-18) vs fp64 PyTorch and vs
the conv_igemm tile with the same wave tiling (same K order: bit-identical outputs): forward with
BN affine / residual / ReLU / APoZ counts (LDS-reduced and direct-atomic paths), strided
downsample convs, ragged M and N, several tiles per workgroup, and the masked data gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

WS = 16  # conv_mfma.hip CFG_WS


def _ref(x, w, sc, sh, stride, relu, res=None):
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double()[:, :, None, None], stride=stride)
    if sc is not None:
        y = y * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
    if res is not None:
        y = y + res.permute(0, 3, 1, 2).double()
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,hw,cin,cout,stride", [(4, 14, 64, 256, 1), (3, 7, 256, 64, 1), (2, 15, 128, 96, 2),
                                                  (8, 4, 32, 128, 1), (5, 28, 96, 36, 1), (300, 1, 512, 1000, 1)])
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_gemm_ws_forward(cuda, B, hw, cin, cout, stride, variant, with_res):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(B * 1000 + cin + cout + variant)
    x = torch.randn(B, hw, hw, cin, generator=g)
    w = torch.randn(cout, cin, generator=g) * (2.0 / cin) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    Ho = (hw - 1) // stride + 1
    res = torch.randn(B, Ho, Ho, cout, generator=g) if with_res else None
    ref = _ref(x, w, sc, sh, stride, True, res)
    dx, dw, dsc, dsh = x.to(cuda), w.to(cuda), sc.to(cuda), sh.to(cuda)
    dres = res.to(cuda) if with_res else None
    apoz = torch.zeros(B, cout, device=cuda)
    out = T.conv_gen(dx, dw, dsc, dsh, True, dres, apoz, 1, stride, 0, WS + variant, 1)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    # same K order as the conv_igemm tile with the same wave tiling: bit-identical
    twin = 4 if variant in (0, 1) else 6
    apoz2 = torch.zeros(B, cout, device=cuda)
    out2 = T.conv_gen(dx, dw, dsc, dsh, True, dres, apoz2, 1, stride, 0, twin, 1)
    assert torch.equal(out, out2)
    assert torch.equal(apoz, apoz2)
    assert torch.equal(apoz.cpu(), (out.cpu() > 0).sum((1, 2)).float())


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_gemm_ws_many_tiles_per_workgroup(cuda, variant):
    """More tiles than workgroups (persistent loop, LDS count buffers of both parities) and a
    NaN in the input (propagates through the NaN-preserving ReLU, counted as not positive)."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(7 + variant)
    B, hw, cin, cout = 16, 56, 64, 256
    x = torch.randn(B, hw, hw, cin, generator=g)
    x[3, 5, 7, 11] = float("nan")
    w = torch.randn(cout, cin, generator=g) * 0.2
    res = torch.randn(B, hw, hw, cout, generator=g)
    ref = _ref(x, w, None, None, 1, True, res)
    apoz = torch.zeros(B, cout, device=cuda)
    out = T.conv_gen(x.to(cuda), w.to(cuda), None, None, True, res.to(cuda), apoz, 1, 1, 0, WS + variant, 1).cpu()
    assert torch.isnan(out[3, 5, 7]).all() and torch.isnan(out).sum() == cout
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert torch.equal(apoz.cpu(), (out > 0).sum((1, 2)).float())


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_gemm_ws_dgrad(cuda, variant, with_res):
    """Stride-1 1x1 data gradient with the ReLU-backward mask and a dense residual gradient."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(11 + variant)
    B, C, N, hw = 3, 128, 160, (14, 10)
    wf = torch.randn(C, N, generator=g)  # forward conv N -> C
    gy = torch.randn(B, hw[0], hw[1], C, generator=g)
    ref = torch.einsum("bhwc,cn->bhwn", gy.double(), wf.double())
    res = torch.randn(B, hw[0], hw[1], N, generator=g) if with_res else None
    if with_res:
        ref = ref + res.double()
    mask = torch.randn(B, hw[0], hw[1], N, generator=g).clamp_min(0)
    ref = torch.where(mask.double() > 0, ref, torch.zeros((), dtype=torch.float64))
    wt = wf.t().contiguous()
    args = (gy.to(cuda), wt.to(cuda), res.to(cuda) if with_res else None, 1, mask.to(cuda), 1, 1, 0, 0, 0, False)
    out = T.conv_gen_bwd(*args, WS + variant, 1)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(out, T.conv_gen_bwd(*args, 4 if variant in (0, 1) else 6, 1))


def test_gemm_ws_rejects_unsupported(cuda):
    from torchpruner_amd import ops
    T = ops.require()
    x = torch.randn(2, 8, 8, 32, device=cuda)
    w3 = torch.randn(64, 9 * 32, device=cuda)
    with pytest.raises(RuntimeError):  # 3x3: not a 1x1 GEMM
        T.conv_gen(x, w3, None, None, True, None, None, 3, 1, 1, WS, 1)
