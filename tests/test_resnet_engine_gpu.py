"""General strided conv (conv_gen: ks 1/3/7, stride 1/2, residual, APoZ counts), NHWC pooling,
and the ResNet forward engine vs the generic hook path (APoZ, config #3)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x_nhwc, w, scale, shift, stride, pad, relu, res=None):
    y = F.conv2d(x_nhwc.permute(0, 3, 1, 2).double(), w.double(), stride=stride, padding=pad)
    y = y * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)
    if res is not None:
        y = y + res.permute(0, 3, 1, 2).double()
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("ks,stride,cin,cout,hw", [(1, 1, 64, 96, 14), (1, 2, 64, 128, 14), (3, 1, 32, 64, 9),
                                                   (3, 2, 64, 64, 15), (7, 2, 4, 64, 38)])
@pytest.mark.parametrize("cfg,splits", [(0, 1), (1, 2), (2, 3), (3, 1), (4, 2), (5, 1), (6, 1)])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_gen(cuda, ks, stride, cin, cout, hw, cfg, splits, with_res):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(ks * 100 + stride * 10 + cfg)
    B, pad = 3, ks // 2
    x = torch.randn(B, hw, hw, cin, generator=g)
    if cin == 4:
        x[..., 3] = 0  # padded stem input
    w = torch.randn(cout, cin, ks, ks, generator=g) * (2.0 / (ks * ks * cin)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    Ho = (hw + 2 * pad - ks) // stride + 1
    res = torch.randn(B, Ho, Ho, cout, generator=g) if with_res else None
    ref = _ref(x, w, sc, sh, stride, pad, True, res)
    wk = w.permute(0, 2, 3, 1).reshape(cout, -1)
    kp = T.conv_gen_k(ks, cin) - wk.shape[1]
    wk = F.pad(wk, (0, kp)).contiguous()
    apoz = torch.zeros(B, cout, device=cuda)
    out = T.conv_gen(x.to(cuda), wk.to(cuda), sc.to(cuda), sh.to(cuda), True, res.to(cuda) if with_res else None,
                     apoz, ks, stride, pad, cfg, splits)
    torch.testing.assert_close(out.cpu(), ref.float(), rtol=1e-4, atol=1e-4)
    # counts of positive outputs: exact except for values within rounding of zero
    cnt_ref = (ref > 0).sum((1, 2)).float()
    assert (apoz.cpu() - cnt_ref).abs().max() <= 2


def test_pools(cuda):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 13, 11, 8, generator=g)
    x[0, 3, 4, 1] = float("nan")
    y = T.maxpool_nhwc(x.to(cuda), 3, 2, 1).cpu()
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, ref, equal_nan=True)
    a = T.avgpool_nhwc(x.nan_to_num().to(cuda)).cpu()
    torch.testing.assert_close(a, x.nan_to_num().mean((1, 2)))


def test_resnet_engine_apoz_matches_generic(cuda):
    import os
    from torchpruner_amd import APoZAttributionMetric, get_resnet_pruning_graph
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_resnet_engine
    from torchpruner_amd.models import resnet50
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 2, 1, 1], num_classes=10, width=32).to(cuda).eval()
    for m in model.modules():  # non-trivial BN statistics
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(12, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (12,), device=cuda)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    ev = [find_best_module_for_attributions(model, m) for m in mods]
    assert maybe_resnet_engine(model, ev, cuda) is not None
    dl = DeviceLoader(x, y, 4)
    fused = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(mods, True)
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        generic = APoZAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(mods, True)
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]
    for a, b in zip(fused, generic):
        assert a.shape == b.shape
        np.testing.assert_allclose(a, b, atol=0.5)  # counts: only values within rounding of 0 may flip
    # the engine's logits match the model's
    eng = maybe_resnet_engine(model, ev, cuda)
    with torch.no_grad():
        torch.testing.assert_close(eng.forward(x), model(x), rtol=2e-3, atol=2e-3)
    assert resnet50 is not None


@pytest.mark.parametrize("which", ["apoz", "taylor", "sensitivity"])
def test_resnet_two_stream_pipeline_bit_identical(cuda, which):
    """ResNet engine runs with two batches in flight (attributions/base.py _BatchPipeline) give
    the one-stream scores bit for bit, ragged last batch included."""
    import os
    from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric, TaylorAttributionMetric,
                                 get_resnet_pruning_graph)
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    torch.manual_seed(2)
    model = ResNet(Bottleneck, [1, 2, 1, 1], num_classes=10, width=32).to(cuda).eval()
    x = torch.randn(22, 3, 64, 64, device=cuda)  # 5 batches of 4 + a ragged 2
    y = torch.randint(0, 10, (22,), device=cuda)
    mods = [m for m, _ in get_resnet_pruning_graph(model)]
    metric = {"apoz": APoZAttributionMetric, "taylor": TaylorAttributionMetric,
              "sensitivity": SensitivityAttributionMetric}[which]
    out = {}
    for env in ("0", "1"):
        old = os.environ.get("TORCHPRUNER_STREAMS")
        os.environ["TORCHPRUNER_STREAMS"] = env
        try:
            m = metric(model, DeviceLoader(x, y, 4), F.cross_entropy, cuda)
            out[env] = m.run_many(mods, True)
            assert m.last_path["path"] == "resnet", m.last_path
        finally:
            if old is None:
                del os.environ["TORCHPRUNER_STREAMS"]
            else:
                os.environ["TORCHPRUNER_STREAMS"] = old
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)
