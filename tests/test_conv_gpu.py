"""Fused conv/GEMM kernels (csrc/kernels/conv_mfma.hip) vs plain PyTorch fp32 references, and
the fused VGG engine vs the generic hook path."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # B, H, W, Cin, Cout
    (4, 32, 32, 64, 64),
    (3, 16, 16, 128, 128),
    (5, 8, 8, 256, 256),
    (6, 4, 4, 512, 512),
    (16, 2, 2, 512, 512),
    (2, 6, 10, 32, 96),
]


def _rand(*shape, gen):
    return torch.randn(*shape, generator=gen)


def _ref_fwd(x_nhwc, w, scale, shift, relu, pool):
    x = x_nhwc.permute(0, 3, 1, 2).double()
    y = F.conv2d(x, w.double(), padding=w.shape[-1] // 2)
    y = y * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)
    if relu:
        y = y.clamp_min(0)
    am = None
    if pool:
        y, idx = F.max_pool2d(y, 2, return_indices=True)
        H = x.shape[2]
        W = x.shape[3]
        ih, iw = idx // W, idx % W
        am = ((ih % 2) * 2 + (iw % 2)).permute(0, 2, 3, 1)
    return y.permute(0, 2, 3, 1).float(), am


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("pool", [False, True])
def test_conv_fwd(cuda, shape, cfg, splits, pool):
    from torchpruner_amd import ops
    T = ops.require()
    B, H, W, Cin, Cout = shape
    g = torch.Generator().manual_seed(hash((shape, cfg)) % 1000)
    x = _rand(B, H, W, Cin, gen=g)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (2.0 / (9 * Cin)) ** 0.5
    scale = _rand(Cout, gen=g).abs() + 0.5
    shift = _rand(Cout, gen=g) * 0.1
    ref, am_ref = _ref_fwd(x, w, scale, shift, True, pool)
    wk = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
    out, am = T.conv_fwd(x.to(cuda), wk.to(cuda), scale.to(cuda), shift.to(cuda), True, pool, 3, cfg, splits)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-4)
    if pool:
        # argmax must point at the max (ties are measure-zero for random data)
        assert (am.cpu().long() == am_ref).float().mean() > 0.999


@pytest.mark.parametrize("B,K,N", [(37, 512, 512), (37, 512, 10), (256, 512, 512), (8, 4096, 96)])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_fwd(cuda, B, K, N, relu):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(B + K + N)
    x = _rand(B, K, gen=g)
    w = _rand(N, K, gen=g) / K ** 0.5
    b = _rand(N, gen=g)
    ref = F.linear(x.double(), w.double(), b.double())
    if relu:
        ref = ref.clamp_min(0)
    for cfg in (0, 2, 3):
        out, _ = T.conv_fwd(x.view(B, 1, 1, K).to(cuda), w.to(cuda), None, b.to(cuda), relu, False, 1, cfg, 2)
        torch.testing.assert_close(out.view(B, N).cpu(), ref.float(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", [0, 2, 3])
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("unpool", [False, True])
def test_conv_dgrad_taylor(cuda, shape, cfg, splits, unpool):
    from torchpruner_amd import ops
    T = ops.require()
    B, H, W, Cin, Cout = shape  # conv maps Cin -> Cout; dgrad goes back to Cin
    g = torch.Generator().manual_seed(7 + hash(shape) % 100)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (1.0 / (9 * Cin)) ** 0.5
    act = torch.relu(_rand(B, H, W, Cin, gen=g))  # post-ReLU activation at the conv input
    bn_scale = _rand(Cin, gen=g).abs() + 0.5
    if unpool:
        gp = _rand(B, H // 2, W // 2, Cout, gen=g)
        am = torch.randint(0, 4, (B, H // 2, W // 2, Cout), generator=g, dtype=torch.uint8)
        gfull = torch.zeros(B, H, W, Cout)
        for q in range(4):
            dy, dx = q // 2, q % 2
            gfull[:, dy::2, dx::2, :] = torch.where(am == q, gp, torch.zeros(()))
    else:
        gfull = _rand(B, H, W, Cout, gen=g)
    # reference: dL/dx of the conv, Taylor of act, masked/scaled grad
    dx = torch.nn.grad.conv2d_input((B, Cin, H, W), w.double(), gfull.permute(0, 3, 1, 2).double(), padding=1)
    dx = dx.permute(0, 2, 3, 1)
    tay_ref = (-(dx * act.double())).sum((1, 2))
    out_ref = torch.where(act > 0, dx * bn_scale.double(), torch.zeros((), dtype=torch.float64))
    wt = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, -1).contiguous()
    tay = torch.zeros(B, Cin, device=cuda)
    gin = (gp if unpool else gfull).to(cuda)
    out = T.conv_dgrad(gin, am.to(cuda) if unpool else None, wt.to(cuda), act.to(cuda), bn_scale.to(cuda), tay,
                       True, 3, cfg, splits)
    torch.testing.assert_close(out.cpu(), out_ref.float(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(tay.cpu(), tay_ref.float(), rtol=1e-4, atol=1e-3)


def test_conv_first(cuda):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(3)
    x = _rand(5, 3, 32, 32, gen=g)
    w = _rand(64, 3, 3, 3, gen=g) * 0.3
    s = _rand(64, gen=g).abs()
    t = _rand(64, gen=g)
    ref = (F.conv2d(x.double(), w.double(), padding=1) * s.double().view(1, -1, 1, 1)
           + t.double().view(1, -1, 1, 1)).clamp_min(0).permute(0, 2, 3, 1)
    out = T.conv_first(x.to(cuda), w.to(cuda), s.to(cuda), t.to(cuda), True)
    torch.testing.assert_close(out.cpu(), ref.float(), rtol=1e-4, atol=1e-4)


def test_nan_propagation(cuda):
    """The pruner's NaN probe relies on NaN surviving conv+ReLU+pool (SURVEY §7.3 hard part 2)."""
    from torchpruner_amd import ops
    T = ops.require()
    x = torch.randn(2, 4, 4, 32)
    x[:, 1, 1, 5] = float("nan")
    w = torch.randn(32, 32 * 9) * 0.1
    out, am = T.conv_fwd(x.to(cuda), w.to(cuda), None, None, True, True, 3, 2, 1)
    assert torch.isnan(out.cpu()[:, 0, 0]).all()  # the window covering the NaN's receptive field


# Bound on max |fused - oracle| / max |oracle| per layer against the fp64 oracle that replays the
# engine's own ReLU masks and pool argmaxes (engine/oracle.py), per pinned kernel family. Measured
# on MI355X (profiles/numerics/taylor_oracle_per_family.txt): F(4x4) <= 1.2e-5 (its +-2 transform
# points amplify rounding ~8x), F(2x2) / implicit GEMM <= 2.5e-6; the bounds leave ~4x headroom.
_COND_BOUND = {"wino4": 5e-5, "wino4_fused": 5e-5, "wino4_m3": 5e-5, "wino2": 1e-5, "wino2_direct": 1e-5, "igemm": 1e-5}


@pytest.mark.parametrize("family", ["wino4", "wino4_fused", "wino2", "wino2_direct", "igemm"])
@pytest.mark.parametrize("split", ["min", "max"])
@pytest.mark.parametrize("mode", ["taylor", "sensitivity"])
def test_engine_scores_match_fp64_oracle(cuda, family, split, mode):
    """Fused VGG16 Taylor / Sensitivity scores (public API, every conv + the two hidden linears)
    against fp64, with every kernel choice pinned to one family (never timed: the result cannot
    depend on the box). Round 3's driver failure (5.8e-4 vs MIOpen's 2.8e-7) was one ReLU-mask /
    pool-argmax decision of one sample in block 6 that fp32 takes differently from fp64 (a
    pre-activation within rounding of 0): every block upstream then differs by ~1e-3 in ANY fp32
    path, MIOpen included on other boxes. So the tight check conditions fp64 on the engine's own
    decisions; the plain-fp64 check is a loose sanity bound."""
    from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.engine.fused_chain import TUNER, family_policy
    from torchpruner_amd.engine.oracle import engine_scores_fp64, flip_violations
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    mods = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1],
                                                                            model.classifier[4]]
    x = torch.randn(48, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (48,), device=cuda)
    B = 16
    eng, idx = maybe_engine(model, [find_best_module_for_attributions(model, m) for m in mods], F.cross_entropy,
                            cuda)
    with TUNER.pinned(family_policy(family, split)):
        if mode == "taylor":
            got = TaylorAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, cuda, signed=True,
                                          reduction="none").run_many(mods, True)
        else:
            got = SensitivityAttributionMetric(model, DeviceLoader(x, y, B), F.cross_entropy, cuda,
                                               reduction="none").run_many(mods, True)
        cond, plain = {b: [] for b in idx}, {b: [] for b in idx}
        flips, totals = {}, {}
        for i in range(0, x.shape[0], B):
            tot = {}
            c, fl = engine_scores_fp64(eng, x[i:i + B], y[i:i + B], conditioned=True, mode=mode, totals=tot)
            for b in fl:
                flips[b] = flips.get(b, 0) + fl[b]
                totals[b] = totals.get(b, 0) + tot[b]
            p, _ = engine_scores_fp64(eng, x[i:i + B], y[i:i + B], conditioned=False, mode=mode)
            for b in idx:
                cond[b].append(c[b])
                plain[b].append(p[b])
    for a, b in zip(got, idx):
        e = torch.cat(cond[b]).numpy()
        err = np.abs(a - e).max() / (np.abs(e).max() + 1e-30)
        ep = torch.cat(plain[b]).numpy()
        am, pm = np.abs(a).mean(0), np.abs(ep).mean(0)  # the unsigned mean reduction
        err_plain = np.abs(am - pm).max() / (pm.max() + 1e-30)
        print(f"{family}/{split} {mode} block {b}: cond {err:.2e} plain(|.| mean) {err_plain:.2e}")
        assert err < _COND_BOUND[family], (b, err)
        assert err_plain < 5e-3, (b, err_plain)
    # decisions (ReLU masks, pool argmaxes) taken differently from fp64 given identical upstream
    # decisions: rare rounding ties only — a systematic mis-decision near 0 fails here
    # (tests/test_oracle.py::test_flip_bound_catches_a_wrong_relu_threshold)
    print(f"{family}/{split} {mode} decision flips per block: {flips} of {totals}")
    assert flip_violations(flips, totals) == {}, flip_violations(flips, totals)


def test_engine_taylor_bit_reproducible(cuda):
    """The fused Taylor path has no float atomics: repeated runs give identical scores."""
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(64, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (64,), device=cuda)
    runs = [TaylorAttributionMetric(model, DeviceLoader(x, y, 32), F.cross_entropy, cuda).run_many(convs, True)
            for _ in range(3)]
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("layer", [1, 5, 12, 14])
def test_engine_shapley_matches_generic_path(cuda, layer):
    """Fused prefix evaluation (pooled-activation masking, fused downstream forward) gives the
    same Shapley values as the reference-style forward_partial path, same permutations."""
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    prunable = [m for m in model.features if isinstance(m, torch.nn.Conv2d)] + [model.classifier[1],
                                                                                 model.classifier[4]]
    module = prunable[layer]
    x = torch.randn(12, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (12,), device=cuda)
    dl = DeviceLoader(x, y, 6)
    import copy
    m64 = copy.deepcopy(model).double().cpu()
    p64 = [m for m in m64.features if isinstance(m, torch.nn.Conv2d)] + [m64.classifier[1], m64.classifier[4]]
    dl64 = DeviceLoader(x.double().cpu(), y.cpu(), 6)
    from torchpruner_amd.engine.fused_chain import TUNER
    res = []
    for backend, mdl, mod, d, dd in (("hip", model, module, cuda, dl), ("torch", model, module, cuda, dl),
                                     ("torch", m64, p64[layer], "cpu", dl64)):
        os.environ["TORCHPRUNER_BACKEND"] = backend
        try:
            np.random.seed(11)
            with TUNER.fixed():  # pinned kernel choices: the fused numbers are the same on any box
                res.append(ShapleyAttributionMetric(mdl, dd, F.cross_entropy, d, sv_samples=2,
                                                    reduction="none").run(mod, find_best_evaluation_module=True))
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
    with torch.no_grad():
        lbar = float(F.cross_entropy(m64(x.double().cpu()), y.cpu()))
    err_fused = np.abs(res[0] - res[2]).max()
    err_generic = np.abs(res[1] - res[2]).max()
    ulps = err_fused / (np.finfo(np.float32).eps * lbar)
    print(f"layer {layer}: fused_err={err_fused:.2e} ({ulps:.0f} fp32 ulps of the mean loss) "
          f"miopen_err={err_generic:.2e}")
    # Shapley values are differences of forward losses (forward = continuous in fp32 rounding:
    # ReLU / max-pool decision flips move a loss by rounding-size amounts only), so the error is
    # bounded in units of fp32 rounding of the loss itself, independent of any other library
    assert ulps < 400, (err_fused, err_generic, lbar)
    # the engine's partial forward itself is exact to fp32 rounding: masked prefix losses
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.utils import find_best_module_for_attributions
    engine, (k,) = maybe_engine(model, [find_best_module_for_attributions(model, module)], F.cross_entropy, cuda)
    zk, _ = engine.forward(x, stop_after=k)
    keep = torch.rand(zk.shape[3], device=cuda) > 0.3
    got = engine.loss_from(k, zk * keep.view(1, 1, 1, -1), y)
    ev64 = find_best_module_for_attributions(m64, p64[layer])
    with torch.no_grad():
        z64 = m64.forward_partial(x.double().cpu(), to_module=ev64)
        shape = (1, -1) + (1,) * (z64.dim() - 2)
        ref = F.cross_entropy(m64.forward_partial(z64 * keep.cpu().double().view(shape), from_module=ev64),
                              y.cpu(), reduction="none")
    torch.testing.assert_close(got.double().cpu(), ref, rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------- Winograd F(2x2,3x3)
WINO_SHAPES = [  # B, H, W, Cin, Cout (staged-region modes: rows for W/2 | 64, images for (H/2)(W/2) | 64)
    (4, 32, 32, 64, 64),
    (3, 64, 32, 32, 64),
    (2, 16, 64, 32, 32),
    (7, 8, 8, 64, 32),
    (3, 16, 16, 128, 256),
    (5, 8, 8, 256, 256),
    (6, 4, 4, 512, 512),
    (16, 2, 2, 512, 512),
    (2, 6, 10, 40, 96),
    (3, 18, 14, 64, 32),
    # ResNet geometries (W/2 = 7, 14, 28 do not divide 64): row-span staged input (X_SPAN),
    # blocks straddling 2-3 images
    (3, 14, 14, 64, 64),
    (2, 28, 28, 32, 64),
    (2, 56, 56, 64, 32),
    (5, 10, 6, 32, 32),
]


@pytest.mark.parametrize("shape", WINO_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("staged", [False, True])
def test_wino_fwd(cuda, shape, splits, pool, staged):
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    B, H, W, Cin, Cout = shape
    g = torch.Generator().manual_seed(11 + hash(shape) % 1000)
    x = _rand(B, H, W, Cin, gen=g)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (2.0 / (9 * Cin)) ** 0.5
    scale = _rand(Cout, gen=g).abs() + 0.5
    shift = _rand(Cout, gen=g) * 0.1
    ref, am_ref = _ref_fwd(x, w, scale, shift, True, pool)
    u = winograd_weights(w.to(cuda))
    out, am = T.conv_wino_fwd(x.to(cuda), u, scale.to(cuda), shift.to(cuda), True, pool, splits, staged)
    torch.testing.assert_close(out.cpu(), ref, rtol=3e-4, atol=3e-4)
    if pool:
        assert (am.cpu().long() == am_ref).float().mean() > 0.999


def test_wino_lds_budget(cuda):
    """The staged Winograd kernels fit two blocks per CU (<= 80 KB of the 160 KB LDS): one more
    __shared__ word would silently halve their occupancy (a 17% headline regression, measured)."""
    from torchpruner_amd import ops
    lds = ops.require().wino_lds_bytes()
    assert 0 < lds <= 80 * 1024, lds


WINO_ODD_SHAPES = [(3, 7, 7, 64, 64), (2, 5, 9, 32, 32), (2, 7, 14, 64, 32), (4, 3, 3, 32, 64), (2, 1, 5, 32, 32)]


@pytest.mark.parametrize("shape", WINO_ODD_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
def test_wino_fwd_odd(cuda, shape, splits):
    """Odd H / W (ResNet-50 layer4's 7x7): a partial last tile row / column, direct loads."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    B, H, W, Cin, Cout = shape
    g = torch.Generator().manual_seed(21 + H * W)
    x = _rand(B, H, W, Cin, gen=g)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (2.0 / (9 * Cin)) ** 0.5
    scale = _rand(Cout, gen=g).abs() + 0.5
    shift = _rand(Cout, gen=g) * 0.1
    ref, _ = _ref_fwd(x, w, scale, shift, True, False)
    u = winograd_weights(w.to(cuda))
    apoz = torch.zeros(B, Cout, device=cuda)
    out, _ = T.conv_wino_fwd(x.to(cuda), u, scale.to(cuda), shift.to(cuda), True, False, splits, True, apoz)
    torch.testing.assert_close(out.cpu(), ref, rtol=3e-4, atol=3e-4)
    if splits == 1:  # the fused APoZ counts see only in-image pixels
        assert torch.equal(apoz.cpu(), (out.cpu() > 0).float().sum((1, 2)))


@pytest.mark.parametrize("shape", WINO_ODD_SHAPES)
@pytest.mark.parametrize("splits", [1, 4])
def test_wino_dgrad_taylor_odd(cuda, shape, splits):
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import taylor_slots, winograd_weights
    T = ops.require()
    B, H, W, Cin, Cout = shape
    g = torch.Generator().manual_seed(7 + H * W)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (1.0 / (9 * Cin)) ** 0.5
    act = torch.relu(_rand(B, H, W, Cin, gen=g))
    bn_scale = _rand(Cin, gen=g).abs() + 0.5
    gfull = _rand(B, H, W, Cout, gen=g)
    dx = torch.nn.grad.conv2d_input((B, Cin, H, W), w.double(), gfull.permute(0, 3, 1, 2).double(), padding=1)
    dx = dx.permute(0, 2, 3, 1)
    tay_ref = (-(dx * act.double())).sum((1, 2))
    out_ref = torch.where(act > 0, dx * bn_scale.double(), torch.zeros((), dtype=torch.float64))
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).to(cuda))
    R = taylor_slots(H, W)
    assert R >= T.wino_taylor_slots(H, W)
    tay = torch.zeros(R, B, Cin, device=cuda)
    out = T.conv_wino_dgrad(gfull.to(cuda), None, ut, act.to(cuda), bn_scale.to(cuda), tay, True, splits, True)
    torch.testing.assert_close(out.cpu(), out_ref.float(), rtol=3e-4, atol=3e-4)
    torch.testing.assert_close(tay.sum(0).cpu(), tay_ref.float(), rtol=3e-4, atol=3e-3)


@pytest.mark.parametrize("shape", WINO_SHAPES)
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("unpool", [False, True])
@pytest.mark.parametrize("staged", [False, True])
def test_wino_dgrad_taylor(cuda, shape, splits, unpool, staged):
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    B, H, W, Cin, Cout = shape
    if Cin % 32:
        pytest.skip("dgrad output channels must be a multiple of 32")
    g = torch.Generator().manual_seed(5 + hash(shape) % 100)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (1.0 / (9 * Cin)) ** 0.5
    act = torch.relu(_rand(B, H, W, Cin, gen=g))
    bn_scale = _rand(Cin, gen=g).abs() + 0.5
    if unpool:
        gp = _rand(B, H // 2, W // 2, Cout, gen=g)
        am = torch.randint(0, 4, (B, H // 2, W // 2, Cout), generator=g, dtype=torch.uint8)
        gfull = torch.zeros(B, H, W, Cout)
        for q in range(4):
            dy, dx = q // 2, q % 2
            gfull[:, dy::2, dx::2, :] = torch.where(am == q, gp, torch.zeros(()))
    else:
        gfull = _rand(B, H, W, Cout, gen=g)
    dx = torch.nn.grad.conv2d_input((B, Cin, H, W), w.double(), gfull.permute(0, 3, 1, 2).double(), padding=1)
    dx = dx.permute(0, 2, 3, 1)
    tay_ref = (-(dx * act.double())).sum((1, 2))
    out_ref = torch.where(act > 0, dx * bn_scale.double(), torch.zeros((), dtype=torch.float64))
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).to(cuda))
    from torchpruner_amd.engine.fused_chain import taylor_slots
    R = taylor_slots(H, W)
    assert R >= T.wino_taylor_slots(H, W)  # the engine may keep extra slots (dense 2x2 layers)
    tay = torch.zeros(R, B, Cin, device=cuda)
    gin = (gp if unpool else gfull).to(cuda)
    out = T.conv_wino_dgrad(gin, am.to(cuda) if unpool else None, ut, act.to(cuda), bn_scale.to(cuda), tay, True,
                            splits, staged)
    torch.testing.assert_close(out.cpu(), out_ref.float(), rtol=3e-4, atol=3e-4)
    torch.testing.assert_close(tay.sum(0).cpu(), tay_ref.float(), rtol=3e-4, atol=3e-3)
    # deterministic: a second launch reproduces the partial slots bit for bit
    tay2 = torch.zeros_like(tay)
    T.conv_wino_dgrad(gin, am.to(cuda) if unpool else None, ut, act.to(cuda), bn_scale.to(cuda), tay2, True,
                      splits, staged)
    assert torch.equal(tay, tay2)


@pytest.mark.parametrize("shape", [(3, 8, 8, 64), (2, 32, 32, 32), (5, 4, 6, 36), (2, 4, 4, 6)])
def test_unpool2_nhwc(cuda, shape):
    """unpool2_nhwc (vectorised path for C % 4 == 0, scalar otherwise) == scatter by argmax."""
    from torchpruner_amd import ops
    T = ops.require()
    B, H, W, C = shape
    g = torch.Generator().manual_seed(11)
    gp = _rand(B, H // 2, W // 2, C, gen=g)
    am = torch.randint(0, 4, (B, H // 2, W // 2, C), generator=g, dtype=torch.uint8)
    ref = torch.zeros(B, H, W, C)
    for q in range(4):
        ref[:, q // 2::2, q % 2::2, :] = torch.where(am == q, gp, torch.zeros(()))
    out = T.unpool2_nhwc(gp.to(cuda), am.to(cuda))
    assert torch.equal(out.cpu(), ref)


def test_wino_dgrad_unpooled_staged_matches_fused_unpool(cuda):
    """The engine's WINO_UNP dgrad (explicit unpool + staged kernel on the dense gradient) gives
    the same output and the same Taylor partial slots, bit for bit, as the staged-unpool kernel
    that rebuilds the full-resolution operand from pooled cells (same operand values, same
    reduction order)."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import taylor_slots, winograd_weights
    T = ops.require()
    B, H, W, Cin, Cout = 4, 16, 16, 64, 128
    g = torch.Generator().manual_seed(21)
    w = _rand(Cout, Cin, 3, 3, gen=g) * (1.0 / (9 * Cin)) ** 0.5
    act = torch.relu(_rand(B, H, W, Cin, gen=g)).to(cuda)
    bn_scale = (_rand(Cin, gen=g).abs() + 0.5).to(cuda)
    gp = _rand(B, H // 2, W // 2, Cout, gen=g).to(cuda)
    am = torch.randint(0, 4, (B, H // 2, W // 2, Cout), generator=g, dtype=torch.uint8).to(cuda)
    ut = winograd_weights(w.flip(2, 3).transpose(0, 1).to(cuda))
    R = taylor_slots(H, W)
    for splits in (1, 2):
        t1, t2 = torch.zeros(R, B, Cin, device=cuda), torch.zeros(R, B, Cin, device=cuda)
        o1 = T.conv_wino_dgrad(gp, am, ut, act, bn_scale, t1, True, splits, True)
        o2 = T.conv_wino_dgrad(T.unpool2_nhwc(gp, am), None, ut, act, bn_scale, t2, True, splits, True)
        assert torch.equal(o1, o2)
        assert torch.equal(t1, t2)


def test_wino_nan_propagation(cuda):
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    x = torch.randn(2, 4, 4, 32)
    x[:, 1, 1, 5] = float("nan")
    u = winograd_weights(torch.randn(32, 32, 3, 3).to(cuda) * 0.1)
    out, am = T.conv_wino_fwd(x.to(cuda), u, None, None, True, True, 1)
    assert torch.isnan(out.cpu()[:, 0, 0]).all()


@pytest.mark.parametrize("staged", [False, True])
def test_first_layer_winograd(cuda, staged):
    """Tiny-Cin first layer: NCHW -> NHWC-8 pad + Winograd == fp64 conv + BN affine + ReLU."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    g = torch.Generator().manual_seed(4)
    x = _rand(6, 3, 32, 32, gen=g)
    w = _rand(64, 3, 3, 3, gen=g) * 0.3
    s = _rand(64, gen=g).abs()
    t = _rand(64, gen=g)
    ref = (F.conv2d(x.double(), w.double(), padding=1) * s.double().view(1, -1, 1, 1)
           + t.double().view(1, -1, 1, 1)).clamp_min(0).permute(0, 2, 3, 1)
    xp = T.nchw_to_nhwc_pad(x.to(cuda), 8)
    assert xp.shape == (6, 32, 32, 8)
    torch.testing.assert_close(xp[..., :3].cpu(), x.permute(0, 2, 3, 1))
    assert torch.count_nonzero(xp[..., 3:]) == 0
    u = winograd_weights(F.pad(w, (0, 0, 0, 0, 0, 5)).to(cuda))
    out, _ = T.conv_wino_fwd(xp, u, s.to(cuda), t.to(cuda), True, False, 1, staged)
    torch.testing.assert_close(out.cpu(), ref.float(), rtol=3e-4, atol=3e-4)


@pytest.mark.parametrize("pool", [False, True])
def test_dense_gemm_2x2_layer_matches_winograd(cuda, pool):
    """2x2-image conv as a dense GEMM (Wbig) == Winograd path: fwd (+pool) and dgrad (+unpool,
    Taylor slots per pixel)."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import (WINO, FusedChainEngine, taylor_slots, winograd_weights)
    T = ops.require()
    g = torch.Generator().manual_seed(21)
    B, C, K = 40, 64, 96
    w = (_rand(K, C, 3, 3, gen=g) * (2.0 / (9 * C)) ** 0.5).to(cuda)
    e = {"w": w.permute(0, 2, 3, 1).reshape(K, -1).contiguous(), "scale": (_rand(K, gen=g).abs() + 0.5).to(cuda),
         "shift": (_rand(K, gen=g) * 0.1).to(cuda), "pool": pool, "u": winograd_weights(w),
         "ut": winograd_weights(w.flip(2, 3).transpose(0, 1).contiguous()),
         "wt": w.flip(2, 3).permute(1, 2, 3, 0).reshape(C, -1).contiguous()}
    eng = FusedChainEngine.__new__(FusedChainEngine)
    h = _rand(B, 2, 2, C, gen=g).to(cuda)
    y_d, am_d = eng._conv_run(T, e, h, FusedChainEngine.DENSE + 0, 2)
    y_w, am_w = eng._conv_run(T, e, h, WINO, 1)
    torch.testing.assert_close(y_d, y_w, rtol=3e-4, atol=3e-4)
    if pool:
        assert (am_d == am_w).float().mean() > 0.999
    # dgrad into a 2x2 activation with C channels
    act = torch.relu(_rand(B, 2, 2, C, gen=g)).to(cuda)
    sc = (_rand(C, gen=g).abs() + 0.5).to(cuda)
    gy = _rand(B, 1 if pool else 2, 1 if pool else 2, K, gen=g).to(cuda)
    am = am_w if pool else None
    R = taylor_slots(2, 2)
    t_d = torch.zeros(R, B, C, device=cuda)
    t_w = torch.zeros(R, B, C, device=cuda)
    o_d = eng._dgrad_run(T, e, gy, am, act, sc, t_d, True, FusedChainEngine.DENSE + 2, 2, sc.repeat(4).contiguous())
    o_w = eng._dgrad_run(T, e, gy, am, act, sc, t_w, True, WINO, 1)
    torch.testing.assert_close(o_d, o_w, rtol=3e-4, atol=3e-4)
    torch.testing.assert_close(t_d.sum(0), t_w.sum(0), rtol=3e-4, atol=3e-4)
    y2, am2 = T.maxpool2_nhwc(y_w if not pool else y_w.new_ones(B, 2, 2, K))
    assert y2.shape == (B, 1, 1, K)


@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("splits", [1, 2])
def test_wino_fwd_apoz_counts(cuda, staged, splits):
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    g = torch.Generator().manual_seed(31)
    B, H, W, C, K = 5, 14, 14, 64, 96
    x = _rand(B, H, W, C, gen=g)
    w = _rand(K, C, 3, 3, gen=g) * (2.0 / (9 * C)) ** 0.5
    sc = _rand(K, gen=g).abs() + 0.5
    sh = _rand(K, gen=g) * 0.1
    ref, _ = _ref_fwd(x, w, sc, sh, True, False)
    apoz = torch.zeros(B, K, device=cuda)
    out, _ = T.conv_wino_fwd(x.to(cuda), winograd_weights(w.to(cuda)), sc.to(cuda), sh.to(cuda), True, False, splits,
                             staged, apoz)
    torch.testing.assert_close(out.cpu(), ref, rtol=3e-4, atol=3e-4)
    cnt = (ref > 0).sum((1, 2)).float()
    assert (apoz.cpu() - cnt).abs().max() <= 2


def _mse_onehot(out, y, reduction="mean"):
    """A non-cross-entropy criterion (MSE to one-hot targets), reference-style signature."""
    return F.mse_loss(out, F.one_hot(y, out.shape[1]).float(), reduction=reduction)


@pytest.mark.parametrize("arch", ["vgg", "resnet"])
@pytest.mark.parametrize("metric", ["taylor", "sensitivity"])
def test_engines_any_criterion(cuda, arch, metric):
    """Gradient metrics with a criterion other than cross-entropy stay on the native engines
    (dL/dlogits through autograd on the logits) and match the fp64 CPU oracle."""
    import copy
    from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import vgg_cifar
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    torch.manual_seed(3)
    if arch == "vgg":
        model = vgg_cifar(11).to(cuda).eval()
        mods = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
        x = torch.randn(32, 3, 32, 32, device=cuda)
    else:
        model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, width=32).to(cuda).eval()
        mods = [b.conv1 for b in model.modules() if isinstance(b, Bottleneck)]
        x = torch.randn(16, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (x.shape[0],), device=cuda)
    cls = TaylorAttributionMetric if metric == "taylor" else SensitivityAttributionMetric
    m = cls(model, DeviceLoader(x, y, 8), _mse_onehot, cuda)
    got = m.run_many(mods, find_best_evaluation_module=True)
    assert m.last_path["path"] == ("fused" if arch == "vgg" else "resnet"), m.last_path
    m64 = copy.deepcopy(model).double().cpu()
    mods64 = [dict(m64.named_modules())[n] for n, mm in model.named_modules() if any(mm is q for q in mods)]
    ref = cls(m64, DeviceLoader(x.double().cpu(), y.cpu(), 8), _mse_onehot, "cpu").run_many(mods64, True)
    for a, e in zip(got, ref):
        assert np.abs(a - e).max() / (np.abs(e).max() + 1e-30) < 5e-3


@pytest.mark.parametrize("arch", ["vgg", "resnet"])
def test_engines_shapley_any_criterion(cuda, arch):
    """Shapley with a non-cross-entropy criterion on the native engines == the fp64 CPU oracle
    (same permutations); per-sample losses from criterion(out, y, reduction="none")."""
    import copy
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import vgg_cifar
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(5)
    if arch == "vgg":
        model = vgg_cifar(11).to(cuda).eval()
        module = [m for m in model.features if isinstance(m, torch.nn.Conv2d)][5]
        x = torch.randn(12, 3, 32, 32, device=cuda)
    else:
        model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=10, width=32).to(cuda).eval()
        module = [b.conv2 for b in model.modules() if isinstance(b, Bottleneck)][2]
        x = torch.randn(8, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (x.shape[0],), device=cuda)
    np.random.seed(3)
    m = ShapleyAttributionMetric(model, DeviceLoader(x, y, 4), _mse_onehot, cuda, sv_samples=2, reduction="none")
    got = m.run(module, find_best_evaluation_module=True)
    assert m.last_path["path"] == ("fused" if arch == "vgg" else "resnet"), m.last_path
    m64 = copy.deepcopy(model).double().cpu()
    name = [n for n, mm in model.named_modules() if mm is module][0]
    np.random.seed(3)
    ref = ShapleyAttributionMetric(m64, DeviceLoader(x.double().cpu(), y.cpu(), 4), _mse_onehot, "cpu", sv_samples=2,
                                   reduction="none").run(dict(m64.named_modules())[name],
                                                         find_best_evaluation_module=True)
    assert np.abs(got - ref).max() / (np.abs(ref).max() + 1e-12) < 2e-3


@pytest.mark.parametrize("pool", [False, True])
def test_fused_first_layer_candidates(cuda, pool):
    """Every first-layer candidate of the fused VGG engine (staged / direct Winograd, VALU direct)
    == fp64 conv + eval BN + ReLU (+ 2x2 max-pool), APoZ counts exact. (A packed-tap implicit-GEMM
    candidate, conv_igemm GEN 2 on a 4-channel input, was measured slower than the staged
    Winograd kernel at B=2048 and dropped.)"""
    from torchpruner_amd import ops
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.engine.fused_chain import WINO, WINO_LDS
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    T = ops.require()
    torch.manual_seed(3)
    model = prunable_vgg16().to(cuda).eval()
    with torch.no_grad():
        bn = model.features[1]
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv = model.features[0]
    eng, _ = maybe_engine(model, [find_best_module_for_attributions(model, conv)], F.cross_entropy, cuda)
    e = eng._pack()["convs"][0]
    e = dict(e, pool=pool)
    x = torch.randn(6, 3, 32, 32, device=cuda)
    ref = F.conv2d(x.double().cpu(), conv.weight.double().cpu(), conv.bias.double().cpu() if conv.bias is not None
                   else None, padding=1)
    ref = F.batch_norm(ref, bn.running_mean.double().cpu(), bn.running_var.double().cpu(), bn.weight.double().cpu(),
                       bn.bias.double().cpu(), False, 0.0, bn.eps)
    pre = torch.relu(ref)
    cnt_ref = (pre > 0).sum((2, 3)).float()
    if pool:
        ref = F.max_pool2d(pre, 2)
    else:
        ref = pre
    ref = ref.permute(0, 2, 3, 1).float()
    cands = [(WINO_LDS, 1), (WINO, 1), (eng.FIRST_DIRECT, 1)]
    for cfg, sp in cands:
        ap = torch.zeros(6, e["scale"].numel(), device=cuda)
        out, _ = eng._first_run(T, e, x, cfg, sp, ap)
        torch.testing.assert_close(out[..., :64].cpu(), ref, rtol=1e-4, atol=1e-4, msg=f"cfg {cfg}")
        assert torch.equal(ap[:, :64].cpu(), cnt_ref), f"cfg {cfg}"
