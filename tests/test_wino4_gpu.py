"""Winograd F(4x4,3x3) kernels (csrc/kernels/wino4.hip) against fp64 PyTorch references:
forward with BN affine + ReLU (+ 2x2 max-pool / argmax, APoZ counts) and the data gradient with
the ReLU-mask / BN-scale output and the Taylor / Sensitivity partials, on the 4/8/16/32-pixel
maps of VGG16-CIFAR, with ragged batches (partial last blocks) and odd channel paddings."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(32, 16, 32, 3), (32, 64, 64, 2), (16, 64, 128, 3), (16, 128, 96, 1), (8, 128, 256, 5), (8, 24, 32, 2),
          (4, 256, 512, 3), (4, 64, 32, 37)]


def _ops():
    from torchpruner_amd import ops
    return ops.require()


def _fwd_ref(x, w, sc, sh):
    y = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), padding=1)
    y = y * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
    return torch.relu(y).permute(0, 2, 3, 1)


@pytest.mark.parametrize("S,C,K,B", SHAPES)
@pytest.mark.parametrize("variant", [0, 2, 3])  # 2: MODE 3 + spread DMA, 3: split points
def test_wino4_forward(cuda, S, C, K, B, variant):
    T = _ops()
    g = torch.Generator(device=cuda).manual_seed(S * 1000 + C + K)
    x = torch.randn(B, S, S, C, device=cuda, generator=g)
    w = torch.randn(K, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)
    sc = torch.rand(K, device=cuda, generator=g) + 0.5
    sh = torch.randn(K, device=cuda, generator=g) * 0.1
    u = T.wino4_weights(w, False, 0, 0)
    apoz = torch.zeros(B, K, device=cuda)
    y, _ = T.conv_wino4_fwd(x, u, sc, sh, True, False, apoz, 1, variant)
    ref = _fwd_ref(x, w, sc, sh)
    err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-5, err
    cnt = (ref > 0).sum((1, 2)).float()
    assert (apoz - cnt).abs().max().item() <= max(2.0, 1e-3 * S * S), (apoz - cnt).abs().max()
    # pooled epilogue
    apoz2 = torch.zeros(B, K, device=cuda)
    yp, am = T.conv_wino4_fwd(x, u, sc, sh, True, True, apoz2, 1, variant)
    r4 = ref.permute(0, 3, 1, 2)
    pooled, idx = F.max_pool2d(r4, 2, return_indices=True)
    errp = ((yp.double() - pooled.permute(0, 2, 3, 1)).abs().max() / pooled.abs().max()).item()
    assert errp < 2e-5, errp
    # argmax byte = (dy << 1) | dx of the window; compare where the window max is unique enough
    H2 = S // 2
    ii = idx.permute(0, 2, 3, 1)
    dy = (ii // S) % 2
    dx = (ii % S) % 2
    want = (dy * 2 + dx).to(torch.uint8)
    top2 = r4.unfold(2, 2, 2).unfold(3, 2, 2).reshape(B, K, H2, H2, 4).sort(-1).values
    clear = ((top2[..., 3] - top2[..., 2]) > 1e-4 * pooled.abs().max()).permute(0, 2, 3, 1) & (pooled.permute(0, 2, 3, 1) > 0)
    assert torch.equal((am & 3)[clear], want[clear])
    assert (apoz2 - cnt).abs().max().item() <= max(2.0, 1e-3 * S * S)


@pytest.mark.parametrize("S,C,K,B", SHAPES)
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("variant", [0, 2, 3])
def test_wino4_dgrad(cuda, S, C, K, B, mode, variant):
    """dgrad of conv(Cin=K -> Cout=C): g (B,S,S,C) -> dL/dact (B,S,S,K) with the W_BWD epilogue."""
    T = _ops()
    Cout, Cin = C, K
    gen = torch.Generator(device=cuda).manual_seed(S * 7 + C * 3 + K)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda, generator=gen) / (3 * Cin ** 0.5)
    go = torch.randn(B, S, S, Cout, device=cuda, generator=gen)
    act = torch.relu(torch.randn(B, S, S, Cin, device=cuda, generator=gen))
    sc = torch.rand(Cin, device=cuda, generator=gen) + 0.5
    ut = T.wino4_weights(w, True, 0, 0)
    R = 2
    tay = torch.zeros(R, B, Cin, device=cuda)
    out = T.conv_wino4_dgrad(go, ut, act, sc, tay, True, mode, 1, variant)
    dx = torch.nn.grad.conv2d_input((B, Cin, S, S), w.double(), go.double().permute(0, 3, 1, 2), padding=1)
    dx = dx.permute(0, 2, 3, 1)
    ref_out = torch.where(act.double() > 0, dx * sc.double(), torch.zeros((), dtype=torch.float64, device=cuda))
    err = ((out.double() - ref_out).abs().max() / ref_out.abs().max()).item()
    assert err < 2e-5, err
    part = dx.abs() if mode else -(dx * act.double())
    ref_t = part.sum((1, 2))
    got_t = tay.double().sum(0)
    errt = ((got_t - ref_t).abs().max() / ref_t.abs().max()).item()
    assert errt < 2e-5, errt
    if S != 32:
        assert tay[1].abs().max().item() == 0.0  # whole images per block: slot 0 only


def test_wino4_deterministic_and_lds_budget(cuda):
    T = _ops()
    x = torch.randn(7, 16, 16, 64, device=cuda)
    w = torch.randn(128, 64, 3, 3, device=cuda) * 0.05
    u = T.wino4_weights(w, False, 0, 0)
    for variant in (0, 2, 3):
        a1, _ = T.conv_wino4_fwd(x, u, None, None, False, False, None, 1, variant)
        a2, _ = T.conv_wino4_fwd(x, u, None, None, False, False, None, 1, variant)
        assert torch.equal(a1, a2)
    for S in (4, 8, 16, 32):
        assert 0 < T.wino4_lds_bytes(S) <= 160 * 1024
        assert 0 < T.wino4_lds_bytes(S, 1) <= 160 * 1024


def test_wino4_rejects_bad_shapes(cuda):
    T = _ops()
    w = torch.randn(32, 8, 3, 3, device=cuda)
    u = T.wino4_weights(w, False, 0, 0)
    with pytest.raises(RuntimeError):
        T.conv_wino4_fwd(torch.randn(2, 12, 12, 8, device=cuda), u, None, None, True, False, None)
    with pytest.raises(RuntimeError):
        T.conv_wino4_fwd(torch.randn(2, 16, 8, 8, device=cuda), u, None, None, True, False, None)


@pytest.mark.parametrize("S,C,K,B", [(32, 64, 64, 3), (16, 128, 96, 2), (8, 256, 64, 5), (4, 512, 64, 7)])
@pytest.mark.parametrize("splits", [2, 4])
@pytest.mark.parametrize("variant", [0, 2, 3])
def test_wino4_split_k(cuda, S, C, K, B, splits, variant):
    """Channel split-K (raw slabs + the deterministic combine) == one K pass, all epilogues."""
    T = _ops()
    import os
    if int(os.environ.get("TP_W4_MODE", "3")) < 2:
        pytest.skip("split-K needs MODE 2/3")
    g = torch.Generator(device=cuda).manual_seed(S + C + splits)
    x = torch.randn(B, S, S, C, device=cuda, generator=g)
    w = torch.randn(K, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)
    sc = torch.rand(K, device=cuda, generator=g) + 0.5
    sh = torch.randn(K, device=cuda, generator=g) * 0.1
    u = T.wino4_weights(w, False, 0, 0)
    for pool in (False, True):
        a1 = torch.zeros(B, K, device=cuda)
        a2 = torch.zeros(B, K, device=cuda)
        y1, m1 = T.conv_wino4_fwd(x, u, sc, sh, True, pool, a1, 1, variant)
        y2, m2 = T.conv_wino4_fwd(x, u, sc, sh, True, pool, a2, splits, variant)
        assert ((y1 - y2).abs().max() / y1.abs().max()).item() < 1e-4
        assert (a1 - a2).abs().max().item() <= 2.0
        if pool:
            agree = ((m1 & 3) == (m2 & 3)).float().mean().item()
            assert agree > 0.999, agree
        ref = _fwd_ref(x, w, sc, sh)
        if not pool:
            assert ((y2.double() - ref).abs().max() / ref.abs().max()).item() < 2e-5
    # dgrad of conv(Cin=K -> Cout=C) with Taylor partials
    go = torch.randn(B, S, S, C, device=cuda, generator=g)
    wd = torch.randn(C, K, 3, 3, device=cuda, generator=g) / (3 * K ** 0.5)
    act = torch.relu(torch.randn(B, S, S, K, device=cuda, generator=g))
    scp = torch.rand(K, device=cuda, generator=g) + 0.5
    ut = T.wino4_weights(wd, True, 0, 0)
    t1, t2 = torch.zeros(2, B, K, device=cuda), torch.zeros(2, B, K, device=cuda)
    o1 = T.conv_wino4_dgrad(go, ut, act, scp, t1, True, 0, 1, variant)
    o2 = T.conv_wino4_dgrad(go, ut, act, scp, t2, True, 0, splits, variant)
    assert ((o1 - o2).abs().max() / o1.abs().max()).item() < 1e-4  # summation order only
    s1, s2 = t1.double().sum(0), t2.double().sum(0)
    assert ((s1 - s2).abs().max() / s1.abs().max()).item() < 1e-4
    o3 = T.conv_wino4_dgrad(go, ut, act, scp, None, True, 0, splits, variant)
    assert torch.equal(o2, o3)  # deterministic combine


@pytest.mark.parametrize("S,C,K,B", [(16, 64, 128, 3), (8, 128, 256, 2), (4, 256, 512, 5), (8, 32, 64, 1)])
@pytest.mark.parametrize("variant", [0, 3])
def test_wino4_dgrad_fused_unpool(cuda, S, C, K, B, variant):
    """The data gradient written unpooled through the previous block's 2x2-pool argmax bytes
    (engine: no separate unpooling pass) == the pooled output followed by unpool2_nhwc, bit for
    bit, with the Taylor partials unchanged."""
    T = _ops()
    Cout, Cin = C, K
    g = torch.Generator(device=cuda).manual_seed(S + C + K + B)
    go = torch.randn(B, S, S, Cout, device=cuda, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda, generator=g) / (3 * Cin ** 0.5)
    act = torch.relu(torch.randn(B, S, S, Cin, device=cuda, generator=g))
    sc = torch.rand(Cin, device=cuda, generator=g) + 0.5
    am = torch.randint(0, 4, (B, S, S, Cin), device=cuda, generator=g, dtype=torch.uint8)
    ut = T.wino4_weights(w, True, 0, 0)
    t1 = torch.zeros(2, B, Cin, device=cuda)
    t2 = torch.zeros(2, B, Cin, device=cuda)
    ref = T.unpool2_nhwc(T.conv_wino4_dgrad(go, ut, act, sc, t1, True, 0, 1, variant), am)
    got = T.conv_wino4_dgrad(go, ut, act, sc, t2, True, 0, 1, variant, am)
    assert got.shape == (B, 2 * S, 2 * S, Cin)
    assert torch.equal(got, ref)
    assert torch.equal(t1, t2)
    with pytest.raises(RuntimeError):  # split-K combines pooled rows: the fused path is one K pass
        T.conv_wino4_dgrad(go, ut, act, sc, None, True, 0, 2, variant, am)


# band geometry (split-points kernel, variant 3): ResNet's 56/28/14/7-pixel maps — whole tile rows
# per block counted across images (28-pixel bands straddle images), partial last tiles at 14 / 7
BAND_SHAPES = [(56, 64, 64, 3), (28, 128, 128, 2), (14, 256, 256, 3), (7, 512, 64, 5), (28, 24, 32, 3),
               (7, 64, 96, 37), (14, 32, 32, 1)]


@pytest.mark.parametrize("S,C,K,B", BAND_SHAPES)
def test_wino4_band_forward(cuda, S, C, K, B):
    T = _ops()
    g = torch.Generator(device=cuda).manual_seed(S * 1000 + C + K + B)
    x = torch.randn(B, S, S, C, device=cuda, generator=g)
    w = torch.randn(K, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)
    sc = torch.rand(K, device=cuda, generator=g) + 0.5
    sh = torch.randn(K, device=cuda, generator=g) * 0.1
    u = T.wino4_weights(w, False, 0, 0)
    apoz = torch.zeros(B, K, device=cuda)
    y, _ = T.conv_wino4_fwd(x, u, sc, sh, True, False, apoz, 1, 3)
    ref = _fwd_ref(x, w, sc, sh)
    err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-5, err
    cnt = (ref > 0).sum((1, 2)).float()
    assert (apoz - cnt).abs().max().item() <= max(2.0, 1e-3 * S * S), (apoz - cnt).abs().max()
    # no pooling, and only the split-points kernel has the band geometry
    with pytest.raises(RuntimeError):
        T.conv_wino4_fwd(x, u, sc, sh, True, True, None, 1, 3)
    with pytest.raises(RuntimeError):
        T.conv_wino4_fwd(x, u, sc, sh, True, False, None, 1, 0)


@pytest.mark.parametrize("S,C,K,B", BAND_SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_wino4_band_dgrad(cuda, S, C, K, B, mode):
    """Band-geometry data gradient: masked output and the Taylor / Sensitivity / masked-|g| partials
    over T.wino4_taylor_slots(S) slots (a band straddling two images writes one slot of each)."""
    T = _ops()
    Cout, Cin = C, K
    gen = torch.Generator(device=cuda).manual_seed(S * 7 + C * 3 + K + mode)
    w = torch.randn(Cout, Cin, 3, 3, device=cuda, generator=gen) / (3 * Cin ** 0.5)
    go = torch.randn(B, S, S, Cout, device=cuda, generator=gen)
    act = torch.relu(torch.randn(B, S, S, Cin, device=cuda, generator=gen))
    sc = torch.rand(Cin, device=cuda, generator=gen) + 0.5
    ut = T.wino4_weights(w, True, 0, 0)
    R = T.wino4_taylor_slots(S)
    assert R >= 1
    tay = torch.zeros(R, B, Cin, device=cuda)
    out = T.conv_wino4_dgrad(go, ut, act, sc, tay, True, mode, 1, 3)
    dx = torch.nn.grad.conv2d_input((B, Cin, S, S), w.double(), go.double().permute(0, 3, 1, 2), padding=1)
    dx = dx.permute(0, 2, 3, 1)
    zero = torch.zeros((), dtype=torch.float64, device=cuda)
    ref_out = torch.where(act.double() > 0, dx * sc.double(), zero)
    err = ((out.double() - ref_out).abs().max() / ref_out.abs().max()).item()
    assert err < 2e-5, err
    part = {0: -(dx * act.double()), 1: dx.abs(), 2: torch.where(act.double() > 0, dx.abs(), zero)}[mode]
    ref_t = part.sum((1, 2))
    errt = ((tay.double().sum(0) - ref_t).abs().max() / ref_t.abs().max()).item()
    assert errt < 2e-5, errt
    # no output: the partials alone
    tay2 = torch.zeros(R, B, Cin, device=cuda)
    T.conv_wino4_dgrad(go, ut, act, sc, tay2, False, mode, 1, 3)
    assert torch.equal(tay2, tay)


@pytest.mark.parametrize("S,C,K,B", [(56, 64, 64, 2), (28, 128, 64, 3), (7, 512, 64, 4)])
def test_wino4_band_split_k(cuda, S, C, K, B):
    T = _ops()
    g = torch.Generator(device=cuda).manual_seed(S + C + 11)
    x = torch.randn(B, S, S, C, device=cuda, generator=g)
    w = torch.randn(K, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)
    sc = torch.rand(K, device=cuda, generator=g) + 0.5
    sh = torch.randn(K, device=cuda, generator=g) * 0.1
    u = T.wino4_weights(w, False, 0, 0)
    a1, a2 = torch.zeros(B, K, device=cuda), torch.zeros(B, K, device=cuda)
    y1, _ = T.conv_wino4_fwd(x, u, sc, sh, True, False, a1, 1, 3)
    y2, _ = T.conv_wino4_fwd(x, u, sc, sh, True, False, a2, 2, 3)
    assert ((y1 - y2).abs().max() / y1.abs().max()).item() < 1e-4
    assert (a1 - a2).abs().max().item() <= 2.0
    assert 0 < T.wino4_lds_bytes(S) <= 80 * 1024  # two blocks per CU
