"""Stream-K launches of the GEN implicit GEMM (conv_mfma.hip launch_gen, cfg | 32): the tiles x
k-slices space cut into one equal range per co-resident block, every cut tile finished by the
fixup launch from its two partial sets. Checked against an fp64 PyTorch reference and against the
data-parallel launch of the same tile config: the fused epilogues (BN affine, residual, ReLU, APoZ
counts, ReLU-backward mask, Taylor partials, BatchNorm statistics) see the same accumulator, the
result is bit-reproducible run to run, and ragged M / N edges are handled."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SK = 32  # conv_mfma.hip CFG_SK


def _sk_cfgs(T, ks, M, N, tay=False):
    cfgs = [c for c in range(7) if T.conv_sk_ws(c, ks, tay, M, N) > 0]
    assert cfgs, f"stream-K applies to no tile config at M={M} N={N}"
    return cfgs


def _fwd_ref(x, w, ks, pad, sc, sh, res, relu):
    cin = x.shape[3]
    w4 = w.double().view(w.shape[0], ks, ks, cin).permute(0, 3, 1, 2)
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w4, padding=pad)
    y = y * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
    if res is not None:
        y = y + res.permute(0, 3, 1, 2).double()
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,hw,cin,cout,ks", [(256, 7, 512, 2048, 1), (256, 14, 256, 1024, 1), (256, 7, 512, 512, 3),
                                              (100, 7, 256, 1000, 1), (512, 7, 96, 164, 3)])
def test_streamk_forward(cuda, B, hw, cin, cout, ks):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(B + hw + cin + cout + ks)
    pad = ks // 2
    x = torch.randn(B, hw, hw, cin, generator=g).to(cuda)
    w = (torch.randn(cout, ks * ks * cin, generator=g) * (2.0 / (ks * ks * cin)) ** 0.5).to(cuda)
    sc = (torch.rand(cout, generator=g) + 0.5).to(cuda)
    sh = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    res = torch.randn(B, hw, hw, cout, generator=g).to(cuda)
    assert w.shape[1] == T.conv_gen_k(ks, cin)
    ref = _fwd_ref(x, w, ks, pad, sc, sh, res, True)
    M = B * hw * hw
    for cfg in _sk_cfgs(T, ks, M, cout):
        ap = torch.zeros(B, cout, device=cuda)
        out = T.conv_gen(x, w, sc, sh, True, res, ap, ks, 1, pad, cfg | SK, 1)
        torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4, msg=lambda m: f"cfg {cfg}: {m}")
        assert torch.equal(ap, (out > 0).sum((1, 2)).float()), cfg
        ap2 = torch.zeros(B, cout, device=cuda)
        again = T.conv_gen(x, w, sc, sh, True, res, ap2, ks, 1, pad, cfg | SK, 1)
        assert torch.equal(out, again) and torch.equal(ap, ap2), f"cfg {cfg}: not reproducible"
        dp = T.conv_gen(x, w, sc, sh, True, res, None, ks, 1, pad, cfg, 1)
        torch.testing.assert_close(out, dp, rtol=1e-4, atol=1e-4)  # K split in two partial sums: rounding order
    # no epilogue at all: the raw accumulator of the fixed-order partial merge
    cfg = _sk_cfgs(T, ks, M, cout)[0]
    raw = T.conv_gen(x, w, None, None, False, None, None, ks, 1, pad, cfg | SK, 1)
    ref_raw = _fwd_ref(x, w, ks, pad, torch.ones_like(sc), torch.zeros_like(sh), None, False)
    torch.testing.assert_close(raw.double(), ref_raw, rtol=1e-4, atol=1e-4)


def test_streamk_falls_back_when_not_applicable(cuda):
    """Too few tiles for the co-resident blocks: the flag runs the data-parallel grid (same bits)."""
    from torchpruner_amd import ops
    T = ops.require()
    x = torch.randn(2, 7, 7, 64, device=cuda)
    w = torch.randn(128, 64, device=cuda) * 0.1
    assert T.conv_sk_ws(0, 1, False, 98, 128) == 0
    a = T.conv_gen(x, w, None, None, True, None, None, 1, 1, 0, 0 | SK, 1)
    b = T.conv_gen(x, w, None, None, True, None, None, 1, 1, 0, 0, 1)
    assert torch.equal(a, b)


@pytest.mark.parametrize("B,hw,c,n", [(256, 7, 2048, 512), (256, 14, 1024, 256), (130, 7, 512, 2044)])
def test_streamk_dgrad_mask_res_taylor(cuda, B, hw, c, n):
    """1x1 stride-1 data gradient: out = mask > 0 ? g @ wt^T + res : 0, and the fused Taylor
    partials of the masked output (tile configs with Taylor slots)."""
    from torchpruner_amd import ops
    T = ops.require()
    gen = torch.Generator().manual_seed(B + c + n)
    g = torch.randn(B, hw, hw, c, generator=gen).to(cuda)
    wt = (torch.randn(n, c, generator=gen) * c ** -0.5).to(cuda)
    res = torch.randn(B, hw, hw, n, generator=gen).to(cuda)
    mask = torch.relu(torch.randn(B, hw, hw, n, generator=gen)).to(cuda)
    v = torch.einsum("bhwc,nc->bhwn", g.double(), wt.double()) + res.double()
    ref = torch.where(mask > 0, v, torch.zeros((), dtype=v.dtype, device=cuda))
    M = B * hw * hw
    for cfg in _sk_cfgs(T, 1, M, n):
        out = T.conv_gen_bwd(g, wt, res, 1, mask, 1, 1, 0, hw, hw, False, cfg | SK, 1, None, 0)
        torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4, msg=lambda m: f"cfg {cfg}: {m}")
    tay_cfgs = [c_ for c_ in range(7) if T.conv_gen_tay_slots(c_, hw * hw) > 0 and T.conv_sk_ws(c_, 1, True, M, n) > 0]
    for cfg in tay_cfgs:
        for mode in (0, 1):
            R = T.conv_gen_tay_slots(cfg, hw * hw)
            t_sk = torch.zeros(R, B, n, device=cuda)
            o_sk = T.conv_gen_bwd(g, wt, None, 1, mask, 1, 1, 0, hw, hw, False, cfg | SK, 1, t_sk, mode)
            t_dp = torch.zeros(R, B, n, device=cuda)
            o_dp = T.conv_gen_bwd(g, wt, None, 1, mask, 1, 1, 0, hw, hw, False, cfg, 1, t_dp, mode)
            torch.testing.assert_close(o_sk, o_dp, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(t_sk.sum(0), t_dp.sum(0), rtol=1e-4, atol=1e-3)


def test_streamk_bn_statistics(cuda):
    """conv_gen_stats: per-tile column sums / sums of squares written by the fixup's epilogue for
    cut tiles and by the main launch for whole ones."""
    from torchpruner_amd import ops
    T = ops.require()
    gen = torch.Generator().manual_seed(5)
    B, hw, cin, cout = 256, 7, 512, 2048
    x = torch.randn(B, hw, hw, cin, generator=gen).to(cuda)
    w = (torch.randn(cout, cin, generator=gen) * cin ** -0.5).to(cuda)
    sh = (torch.randn(cout, generator=gen) * 0.1).to(cuda)
    for cfg in _sk_cfgs(T, 1, B * hw * hw, cout):
        y, part = T.conv_gen_stats(x, w, sh, 1, 1, 0, cfg | SK)
        y0, part0 = T.conv_gen_stats(x, w, sh, 1, 1, 0, cfg)
        torch.testing.assert_close(y, y0, rtol=1e-5, atol=1e-5)
        assert part.shape == part0.shape
        torch.testing.assert_close(part.sum(0), part0.sum(0), rtol=1e-6, atol=1e-3)
        yd = y.double().reshape(-1, cout)
        torch.testing.assert_close(part.sum(0)[0], yd.sum(0), rtol=1e-4, atol=1e-3)  # fp32 in-tile sums
        torch.testing.assert_close(part.sum(0)[1], (yd * yd).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("which", ["apoz", "taylor"])
def test_resnet_engine_with_streamk_pinned(cuda, which):
    """The ResNet engine with every conv that has a stream-K candidate pinned to it gives the scores
    of the same engine pinned to the data-parallel tile configs (APoZ counts up to decisions within
    rounding of 0; Taylor to fp32 rounding), and stream-K really ran."""
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine.fused_chain import CFG_SK, TUNER
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    import numpy as np
    torch.manual_seed(3)
    model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, width=32).to(cuda).eval()
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_var.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.1, 0.1)
    x = torch.randn(32, 3, 224, 224, device=cuda)
    y = torch.randint(0, 10, (32,), device=cuda)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    metric = {"apoz": APoZAttributionMetric, "taylor": TaylorAttributionMetric}[which]
    used = []

    def sk_policy(key, cands, M, N, K):
        sk = [c for c in cands if 0 <= c[0] and c[0] & CFG_SK and c[0] < CFG_SK + 7]
        if sk:
            used.append(key)
            return sk[0]
        return None

    def dp_policy(key, cands, M, N, K):
        dp = [c for c in cands if 0 <= c[0] <= 6 and c[1] == 1]
        return dp[0] if dp else None

    out = {}
    for name, pol in (("sk", sk_policy), ("dp", dp_policy)):
        with TUNER.pinned(pol):
            m = metric(model, DeviceLoader(x, y, 32), F.cross_entropy, cuda)
            out[name] = m.run_many(mods, True)
            assert m.last_path["path"] == "resnet", m.last_path
    assert used, "no conv had a stream-K candidate"
    for a, b in zip(out["sk"], out["dp"]):
        if which == "apoz":
            np.testing.assert_allclose(a, b, atol=0.5)
        else:
            np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-3 * float(np.abs(b).max()))
