"""Opt-in bf16 operands (conv_igemm BF variants: v_mfma_f32_32x32x16_bf16, fp32 accumulation)
against fp64 references: exact-product parity on bf16-rounded operands, bf16 tolerance against
the unrounded op, and the fused engine's Taylor scores under ``compute_dtype=torch.bfloat16``
(rank agreement with the exact fp32 engine, Spearman >= 0.99 per layer)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    from torchpruner_amd import ops
    return ops.require()


def _bf(t):
    return t.bfloat16().double()


@pytest.mark.parametrize("cfg", [256, 258, 259])
@pytest.mark.parametrize("pool", [False, True])
def test_bf16_conv_fwd(cuda, cfg, pool):
    T = _ops()
    g = torch.Generator(device=cuda).manual_seed(cfg + pool)
    B, S, C, K = 3, 16, 64, 96
    x = torch.randn(B, S, S, C, device=cuda, generator=g)
    w = torch.randn(K, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)
    sc = torch.rand(K, device=cuda, generator=g) + 0.5
    sh = torch.randn(K, device=cuda, generator=g) * 0.1
    wk = w.permute(0, 2, 3, 1).reshape(K, 9 * C).contiguous()
    y, am = T.conv_fwd(x, wk, sc, sh, True, pool, 3, cfg, 1, None)

    def ref(xx, ww):
        r = F.conv2d(xx.permute(0, 3, 1, 2), ww, padding=1) * sc.double().view(1, -1, 1, 1) + \
            sh.double().view(1, -1, 1, 1)
        r = torch.relu(r)
        return (F.max_pool2d(r, 2) if pool else r).permute(0, 2, 3, 1)

    exact = ref(_bf(x), _bf(w))  # the same bf16-rounded operands, fp64 products
    err = ((y.double() - exact).abs().max() / exact.abs().max()).item()
    assert err < 1e-5, err
    loose = ref(x.double(), w.double())
    err2 = ((y.double() - loose).abs().max() / loose.abs().max()).item()
    assert err2 < 2e-2, err2


@pytest.mark.parametrize("cfg", [256, 259])
@pytest.mark.parametrize("unpool", [False, True])
def test_bf16_conv_dgrad(cuda, cfg, unpool):
    T = _ops()
    g = torch.Generator(device=cuda).manual_seed(7 + cfg + unpool)
    B, S, Cin, Cout = 2, 16, 64, 64
    w = torch.randn(Cout, Cin, 3, 3, device=cuda, generator=g) / (3 * Cin ** 0.5)
    act = torch.relu(torch.randn(B, S, S, Cin, device=cuda, generator=g))
    sc = torch.rand(Cin, device=cuda, generator=g) + 0.5
    wt = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, 9 * Cout).contiguous()
    if unpool:
        full = torch.randn(B, Cout, S, S, device=cuda, generator=g)
        pooled, idx = F.max_pool2d(full, 2, return_indices=True)
        gp = torch.randn_like(pooled)
        go = F.max_unpool2d(gp, idx, 2, output_size=(S, S)).permute(0, 2, 3, 1).contiguous()
        ii = idx.permute(0, 2, 3, 1)
        am = (((ii // S) % 2) * 2 + (ii % S) % 2).to(torch.uint8).contiguous()
        gin, gam = gp.permute(0, 2, 3, 1).contiguous(), am
    else:
        go = torch.randn(B, S, S, Cout, device=cuda, generator=g)
        gin, gam = go, None
    tay = torch.zeros(B, Cin, device=cuda)
    out = T.conv_dgrad(gin, gam, wt, act, sc, tay, True, 3, cfg, 1, tay_mode=0)

    def ref(gg, ww):
        dx = torch.nn.grad.conv2d_input((B, Cin, S, S), ww, gg.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
        o = torch.where(act.double() > 0, dx * sc.double(), torch.zeros((), dtype=torch.float64, device=cuda))
        return o, (-(dx * act.double())).sum((1, 2))

    o_ex, t_ex = ref(_bf(go), _bf(w))
    assert ((out.double() - o_ex).abs().max() / o_ex.abs().max()).item() < 1e-5
    assert ((tay.double() - t_ex).abs().max() / t_ex.abs().max()).item() < 1e-4
    o_l, _ = ref(go.double(), w.double())
    assert ((out.double() - o_l).abs().max() / o_l.abs().max()).item() < 2e-2


def test_bf16_engine_taylor_ranks_match_fp32(cuda):
    from scipy.stats import spearmanr

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine.fused_chain import CFG_BF16, TUNER, WINO_BF, WINO_BF_UNP
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(256, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (256,), device=cuda)
    dl = DeviceLoader(x, y, 128)
    fp = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(convs, True)
    mb = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda, compute_dtype=torch.bfloat16)
    bf = mb.run_many(convs, True)
    assert mb.last_path["path"] == "fused", mb.last_path
    assert any(isinstance(v, tuple) and (v[0] >= CFG_BF16 or v[0] in (WINO_BF, WINO_BF_UNP))
               for v in TUNER.cache.values())
    for k, (a, b) in enumerate(zip(bf, fp)):
        assert np.isfinite(a).all()
        rho = spearmanr(a, b).correlation
        assert rho >= 0.99, (k, rho)
        assert np.abs(a - b).max() / np.abs(b).max() < 5e-2, k


@pytest.mark.parametrize("family", ["wino2_bf16", "igemm"])
def test_bf16_engine_family_pinned(cuda, family):
    """Each bf16 kernel family pinned in turn (bf16 F(2x2) Winograd with plain bf16-rounded V — the
    hi/lo split is the env-gated TP_WINO_BF_SPLIT path, not tested here — and the bf16 implicit
    GEMM) gives Taylor scores that rank like the fp32 ones; the pinned family really ran."""
    from scipy.stats import spearmanr

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import invalidate
    from torchpruner_amd.engine.fused_chain import CFG_BF16, TUNER, WINO_BF, WINO_BF_UNP, family_policy
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(1)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(128, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (128,), device=cuda)
    fp = TaylorAttributionMetric(model, DeviceLoader(x, y, 64), F.cross_entropy, cuda).run_many(convs, True)
    invalidate(model)
    with TUNER.pinned(family_policy(family)):
        mb = TaylorAttributionMetric(model, DeviceLoader(x, y, 64), F.cross_entropy, cuda,
                                     compute_dtype=torch.bfloat16)
        bf = mb.run_many(convs, True)
        kinds = {v[0] for v in TUNER.cache.values() if isinstance(v, tuple)}
    invalidate(model)
    assert mb.last_path["path"] == "fused", mb.last_path
    if family == "wino2_bf16":
        assert kinds & {WINO_BF, WINO_BF_UNP}, kinds
    else:
        assert any(k >= CFG_BF16 for k in kinds) and not kinds & {WINO_BF, WINO_BF_UNP}, kinds
    rho = []
    for a, b in zip(bf, fp):
        assert np.isfinite(a).all()
        rho.append(spearmanr(a, b).correlation)
    # random-init model, 128 images: near-tied scores (the trained headline teacher ranks at
    # >= 0.9999 in bench.py's bf16 extra)
    assert min(rho) >= 0.98, np.round(rho, 5)


def test_shapley_fp32_after_bf16_on_one_engine(cuda):
    """A bf16 Shapley run must not leave captured graphs / static buffers that a later fp32 run on
    the same engine replays: fp32 after bf16 == a fresh fp32 run, bit for bit."""
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import invalidate
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(2)
    model = prunable_vgg16().to(cuda).eval()
    module = [m for m in model.features if isinstance(m, torch.nn.Conv2d)][8]
    x = torch.randn(24, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (24,), device=cuda)

    def run(dtype):
        np.random.seed(4)
        m = ShapleyAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, cuda, sv_samples=2,
                                     compute_dtype=dtype)
        out = m.run(module, find_best_evaluation_module=True)
        assert m.last_path["path"] == "fused", m.last_path
        return out

    invalidate(model)
    fresh = run(None)
    invalidate(model)
    bf = run(torch.bfloat16)
    after = run(None)
    np.testing.assert_array_equal(after, fresh)
    assert not np.array_equal(bf, fresh)  # the bf16 run really used bf16 operands
