"""conv_gen_bwd (ResNet backward-engine data gradients) vs torch.nn.grad.conv2d_input in fp64:
transposed strided convs (3x3/s2, 1x1/s2, parity-ordered rows and odd sizes), stride-1 1x1 and
flipped 3x3, residual adds (dense and stride-2 scattered) and ReLU-backward masks."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dgrad_ref(g, wf, in_hw, stride, pad):
    """fp64 dL/dx of y = conv2d(x, wf) for NHWC g; returns NHWC."""
    B, N = g.shape[0], wf.shape[1]
    gi = torch.nn.grad.conv2d_input((B, N) + tuple(in_hw), wf.double(), g.permute(0, 3, 1, 2).double(),
                                    stride=stride, padding=pad)
    return gi.permute(0, 2, 3, 1)


@pytest.mark.parametrize("ks,stride,C,N,in_hw", [(3, 2, 64, 32, (16, 16)), (3, 2, 32, 64, (15, 13)),
                                                 (1, 2, 64, 32, (14, 14)), (1, 2, 32, 32, (9, 7)),
                                                 (3, 1, 32, 64, (10, 12))])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("with_mask", [False, True])
def test_conv_gen_bwd_transposed(cuda, ks, stride, C, N, in_hw, cfg, with_mask):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(ks * 7 + stride + cfg)
    B, pad = 3, ks // 2
    wf = torch.randn(C, N, ks, ks, generator=g)  # forward conv N -> C
    H = (in_hw[0] + 2 * pad - ks) // stride + 1
    W = (in_hw[1] + 2 * pad - ks) // stride + 1
    gy = torch.randn(B, H, W, C, generator=g)
    ref = _dgrad_ref(gy, wf, in_hw, stride, pad)
    mask = torch.randn(B, in_hw[0], in_hw[1], N, generator=g).clamp_min(0) if with_mask else None
    if mask is not None:
        ref = torch.where(mask.double() > 0, ref, torch.zeros((), dtype=torch.float64))
    wt = wf.permute(1, 2, 3, 0).reshape(N, ks * ks * C).contiguous()
    out = T.conv_gen_bwd(gy.to(cuda), wt.to(cuda), None, 1, mask.to(cuda) if mask is not None else None,
                         ks, stride, pad, in_hw[0], in_hw[1], True, cfg, 1)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("ks", [1, 3])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("res_stride", [0, 1, 2])
def test_conv_gen_bwd_stride1_res(cuda, ks, splits, res_stride):
    """Stride-1 dgrad as a forward conv (flipped taps) + residual gradient + ReLU mask: the
    bottleneck conv1 dgrad that merges the identity / downsample gradient."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(ks * 10 + splits + res_stride)
    B, C, N, hw = 2, 64, 96, (14, 10)
    pad = ks // 2
    wf = torch.randn(C, N, ks, ks, generator=g)
    gy = torch.randn(B, hw[0], hw[1], C, generator=g)
    ref = _dgrad_ref(gy, wf, hw, 1, pad)
    res = None
    if res_stride:
        rh, rw = -(-hw[0] // res_stride), -(-hw[1] // res_stride)
        res = torch.randn(B, rh, rw, N, generator=g)
        full = torch.zeros(B, hw[0], hw[1], N, dtype=torch.float64)
        full[:, ::res_stride, ::res_stride] = res.double()
        ref = ref + full
    mask = torch.randn(B, hw[0], hw[1], N, generator=g).clamp_min(0)
    ref = torch.where(mask.double() > 0, ref, torch.zeros((), dtype=torch.float64))
    wt = wf.flip(2, 3).permute(1, 2, 3, 0).reshape(N, ks * ks * C).contiguous()
    out = T.conv_gen_bwd(gy.to(cuda), wt.to(cuda), res.to(cuda) if res is not None else None, max(res_stride, 1),
                         mask.to(cuda), ks, 1, pad, 0, 0, False, 2, splits)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cfg", [0, 3])
def test_conv_gen_bwd_transposed_res(cuda, cfg):
    """Strided first conv of a v1 block (3x3/s2 dgrad) merging a stride-2 downsample gradient."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(3 + cfg)
    B, C, N, hw = 2, 32, 64, (12, 10)
    wf = torch.randn(C, N, 3, 3, generator=g)
    gy = torch.randn(B, 6, 5, C, generator=g)
    res = torch.randn(B, 6, 5, N, generator=g)
    mask = torch.randn(B, hw[0], hw[1], N, generator=g).clamp_min(0)
    ref = _dgrad_ref(gy, wf, hw, 2, 1)
    full = torch.zeros(B, hw[0], hw[1], N, dtype=torch.float64)
    full[:, ::2, ::2] = res.double()
    ref = torch.where(mask.double() > 0, ref + full, torch.zeros((), dtype=torch.float64))
    wt = wf.permute(1, 2, 3, 0).reshape(N, 9 * C).contiguous()
    out = T.conv_gen_bwd(gy.to(cuda), wt.to(cuda), res.to(cuda), 2, mask.to(cuda), 3, 2, 1, hw[0], hw[1], True,
                         cfg, 1)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-4, atol=1e-4)


def test_conv_gen_bwd_shape_checks(cuda):
    from torchpruner_amd import ops
    T = ops.require()
    gy = torch.zeros(1, 4, 4, 32, device=cuda)
    with pytest.raises(RuntimeError):
        T.conv_gen_bwd(gy, torch.zeros(8, 9 * 32, device=cuda), None, 1, None, 3, 2, 1, 9, 9, True, 0, 1)
    with pytest.raises(RuntimeError):
        T.conv_gen_bwd(gy, torch.zeros(8, 32, device=cuda), None, 1, None, 3, 1, 1, 0, 0, False, 0, 1)


def _resnet(kind, cuda, prune=False):
    import numpy as np
    from torchpruner_amd import Pruner, get_resnet_pruning_graph
    from torchpruner_amd.models.resnet import BasicBlock, Bottleneck, ResNet
    torch.manual_seed(0)
    block = Bottleneck if kind == "bottleneck" else BasicBlock
    model = ResNet(block, [1, 2, 1, 1], num_classes=10, width=32).to(cuda).eval()
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    if prune:
        rng = np.random.RandomState(0)
        pruner = Pruner(model, (3, 64, 64), cuda)
        for module, cascade in get_resnet_pruning_graph(model):
            n = module.weight.shape[0]
            pruner.prune_model(module, rng.choice(n, int(n * 0.3) + 1, replace=False), cascade)
    return model


# BasicBlock's evaluation module is its shared ReLU (registered between bn1 and conv2, reused
# after the residual add), which the engine deliberately does not score: bottlenecks only
@pytest.mark.parametrize("kind,prune", [("bottleneck", False), ("bottleneck", True)])
def test_resnet_engine_grad_metrics_match_fp64(cuda, kind, prune):
    """Taylor (abs / signed) and Sensitivity on the ResNet backward engine vs an fp64 CPU
    oracle of the same attribution (generic hook path)."""
    import copy
    import os
    import numpy as np
    from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_resnet_engine
    from torchpruner_amd.utils import find_best_module_for_attributions
    model = _resnet(kind, cuda, prune)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    ev = [find_best_module_for_attributions(model, m) for m in mods]
    assert maybe_resnet_engine(model, ev, cuda, grad=True) is not None
    x = torch.randn(8, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    m64 = copy.deepcopy(model).double().cpu()
    mods64 = [m for m, _ in get_resnet_pruning_graph(m64)]
    cases = [(TaylorAttributionMetric, {}, "mean"), (TaylorAttributionMetric, {"signed": True}, "none"),
             (SensitivityAttributionMetric, {}, "mean")]
    for cls, kw, red in cases:
        got = cls(model, DeviceLoader(x, y, 4), F.cross_entropy, cuda, reduction=red, **kw).run_many(mods, True)
        os.environ["TORCHPRUNER_BACKEND"] = "torch"
        try:
            ref = cls(m64, DeviceLoader(x.double().cpu(), y.cpu(), 4), F.cross_entropy, "cpu", reduction=red,
                      **kw).run_many(mods64, True)
        finally:
            del os.environ["TORCHPRUNER_BACKEND"]
        for m, a, r in zip(mods, got, ref):
            assert a.shape == r.shape and a.shape[-1] == m.weight.shape[0]
            err = np.abs(a - r).max() / (np.abs(r).max() + 1e-30)
            assert err < 5e-3, (cls.__name__, kw, red, m, err)


def test_resnet_engine_grad_scores_deterministic(cuda):
    import numpy as np
    from torchpruner_amd import TaylorAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import DeviceLoader
    model = _resnet("bottleneck", cuda)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    x = torch.randn(8, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    runs = [TaylorAttributionMetric(model, DeviceLoader(x, y, 4), F.cross_entropy, cuda).run_many(mods, True)
            for _ in range(2)]
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("prune", [False, True])
def test_resnet_engine_shapley_matches_fp64(cuda, prune):
    """Shapley prefix evaluations through the ResNet engine (masked block-internal activation,
    rest of the block with its residual, remaining blocks) vs the forward_partial path in fp64."""
    import copy
    import os
    import numpy as np
    from torchpruner_amd import ShapleyAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_resnet_engine
    from torchpruner_amd.utils import find_best_module_for_attributions
    model = _resnet("bottleneck", cuda, prune)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    m64 = copy.deepcopy(model).double().cpu()
    mods64 = [m for m, _ in get_resnet_pruning_graph(m64)]
    x = torch.randn(6, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (6,), device=cuda)
    for li in (0, 3, len(mods) - 1):
        ev = find_best_module_for_attributions(model, mods[li])
        assert maybe_resnet_engine(model, [ev], cuda, grad=True) is not None
        res = []
        for backend, mdl, mod, d, xx, yy in (("hip", model, mods[li], cuda, x, y),
                                             ("torch", m64, mods64[li], "cpu", x.double().cpu(), y.cpu())):
            os.environ["TORCHPRUNER_BACKEND"] = backend
            try:
                np.random.seed(7)
                res.append(ShapleyAttributionMetric(mdl, DeviceLoader(xx, yy, 3), F.cross_entropy, d, sv_samples=2,
                                                    reduction="none").run(mod, find_best_evaluation_module=True))
            finally:
                del os.environ["TORCHPRUNER_BACKEND"]
        assert res[0].shape == res[1].shape == (6, mods[li].weight.shape[0])
        scale = np.abs(res[1]).max() + 1e-12
        assert np.abs(res[0] - res[1]).max() / scale < 2e-2, (li, np.abs(res[0] - res[1]).max(), scale)


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 5, 6])
@pytest.mark.parametrize("B,hw,C,N", [(4, 7, 128, 64), (3, 14, 64, 96), (2, 28, 32, 64), (2, 56, 64, 32)])
@pytest.mark.parametrize("tay_mode", [0, 1])
def test_conv_gen_bwd_taylor_partials(cuda, cfg, B, hw, C, N, tay_mode):
    """1x1 dgrad with the Taylor / Sensitivity partials fused into the LDS epilogue (EPI_FWD_TAY):
    the (R, B, N) slots sum to the fp64 reduction of the masked output, the output itself is
    bit-identical to the same config without partials, and images spanning tiles get one slot
    per tile (deterministic: no atomics)."""
    from torchpruner_amd import ops
    T = ops.require()
    R = T.conv_gen_tay_slots(cfg, hw * hw)
    if R == 0:
        pytest.skip("tile spans more than 4 images")
    g = torch.Generator().manual_seed(cfg * 7 + hw + tay_mode)
    wf = torch.randn(C, N, generator=g)  # forward 1x1 conv N -> C
    gy = torch.randn(B, hw, hw, C, generator=g)
    mask = torch.randn(B, hw, hw, N, generator=g).clamp_min(0)
    ref = torch.einsum("bhwc,cn->bhwn", gy.double(), wf.double())
    ref = torch.where(mask.double() > 0, ref, torch.zeros((), dtype=torch.float64))
    tay_ref = ref.abs().sum((1, 2)) if tay_mode else (-(ref * mask.double())).sum((1, 2))
    wt = wf.t().contiguous()
    args = (gy.to(cuda), wt.to(cuda), None, 1, mask.to(cuda), 1, 1, 0, 0, 0, False, cfg, 1)
    tay = torch.zeros(R, B, N, device=cuda)
    out = T.conv_gen_bwd(*args, tay, tay_mode)
    assert torch.equal(out, T.conv_gen_bwd(*args))
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(tay.sum(0).cpu().double(), tay_ref, rtol=1e-4, atol=1e-3)
    tay2 = torch.zeros_like(tay)
    T.conv_gen_bwd(*args, tay2, tay_mode)
    assert torch.equal(tay, tay2)  # deterministic


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 5, 6])
@pytest.mark.parametrize("B,in_hw,C,N", [(3, 14, 64, 32), (2, 28, 32, 64), (2, 56, 64, 32), (5, 8, 32, 32)])
@pytest.mark.parametrize("tay_mode", [0, 1])
def test_conv_gen_bwd_transposed_taylor_partials(cuda, cfg, B, in_hw, C, N, tay_mode):
    """Strided 3x3 dgrad (transposed implicit GEMM, parity row order) with the Taylor / Sensitivity
    partials in its LDS epilogue: one slot range per stride phase, the (4R, B, N) slots sum to the
    fp64 reduction of the masked output, the output is bit-identical to the run without partials,
    and the slots are deterministic."""
    from torchpruner_amd import ops
    T = ops.require()
    R = 4 * T.conv_gen_tay_slots(cfg, in_hw * in_hw // 4)
    if R == 0:
        pytest.skip("tile spans more than 4 (phase, image) row groups")
    g = torch.Generator().manual_seed(cfg * 11 + in_hw + tay_mode)
    wf = torch.randn(C, N, 3, 3, generator=g)  # forward conv N -> C, 3x3 stride 2 pad 1
    H = (in_hw + 2 - 3) // 2 + 1
    gy = torch.randn(B, H, H, C, generator=g)
    mask = torch.randn(B, in_hw, in_hw, N, generator=g).clamp_min(0)
    ref = _dgrad_ref(gy, wf, (in_hw, in_hw), 2, 1)
    ref = torch.where(mask.double() > 0, ref, torch.zeros((), dtype=torch.float64))
    tay_ref = ref.abs().sum((1, 2)) if tay_mode else (-(ref * mask.double())).sum((1, 2))
    wt = wf.permute(1, 2, 3, 0).reshape(N, 9 * C).contiguous()
    args = (gy.to(cuda), wt.to(cuda), None, 1, mask.to(cuda), 3, 2, 1, in_hw, in_hw, True, cfg, 1)
    tay = torch.zeros(R, B, N, device=cuda)
    out = T.conv_gen_bwd(*args, tay, tay_mode)
    assert torch.equal(out, T.conv_gen_bwd(*args))
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(tay.sum(0).cpu().double(), tay_ref, rtol=1e-4, atol=1e-3)
    tay2 = torch.zeros_like(tay)
    T.conv_gen_bwd(*args, tay2, tay_mode)
    assert torch.equal(tay, tay2)


def test_conv_gen_bwd_taylor_partials_rejects_unsupported(cuda):
    """Odd output sizes (no parity row order) and transposed 1x1 dgrads take no partials."""
    from torchpruner_amd import ops
    T = ops.require()
    gy = torch.randn(2, 4, 4, 32, device=cuda)
    wt3 = torch.randn(32, 9 * 32, device=cuda)
    wt1 = torch.randn(32, 32, device=cuda)
    tay = torch.zeros(64, 2, 32, device=cuda)
    with pytest.raises(RuntimeError):  # 7x7 from 4x4: odd
        T.conv_gen_bwd(gy, wt3, None, 1, torch.ones(2, 7, 7, 32, device=cuda), 3, 2, 1, 7, 7, True, 2, 1, tay, 0)
    with pytest.raises(RuntimeError):
        T.conv_gen_bwd(gy, wt1, None, 1, torch.ones(2, 8, 8, 32, device=cuda), 1, 2, 0, 8, 8, True, 2, 1, tay, 0)
