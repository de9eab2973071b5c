"""Native training convolutions (finetune half of config #5): weight-gradient kernel (K3) vs
torch.nn.grad.conv2d_weight in fp64, and the native-conv autograd path vs PyTorch autograd on
pruned (odd-width) ResNets and VGG."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ks,stride,Cin,Cout,hw", [(1, 1, 64, 96, (14, 14)), (1, 1, 36, 40, (7, 9)), (1, 2, 32, 64, (15, 13)),
                                                   (3, 1, 36, 52, (10, 12)), (3, 2, 64, 32, (16, 16)),
                                                   (7, 2, 4, 64, (30, 30))])
@pytest.mark.parametrize("cfg", [0, 1, 2])
@pytest.mark.parametrize("splits", [1, 7])
def test_conv_wgrad(cuda, ks, stride, Cin, Cout, hw, cfg, splits):
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(ks * 31 + stride * 7 + cfg + splits)
    B, pad = 3, ks // 2
    x = torch.randn(B, hw[0], hw[1], Cin, generator=g)
    Ho, Wo = (hw[0] + 2 * pad - ks) // stride + 1, (hw[1] + 2 * pad - ks) // stride + 1
    gy = torch.randn(B, Ho, Wo, Cout, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (Cout, Cin, ks, ks),
                                      gy.permute(0, 3, 1, 2).double(), stride=stride, padding=pad)
    dw = T.conv_wgrad(gy.to(cuda), x.to(cuda), ks, stride, pad, cfg, splits).cpu()
    assert dw.shape == (Cout, -(-ks * ks * Cin // 32) * 32)
    assert (dw[:, ks * ks * Cin:] == 0).all()
    got = dw[:, :ks * ks * Cin].view(Cout, ks, ks, Cin).permute(0, 3, 1, 2)
    torch.testing.assert_close(got.double(), ref, rtol=1e-4, atol=1e-3)


def _grads(model):
    return [p.grad.detach().double().cpu().clone() for p in model.parameters()]


def _step_grads(model, x, y, native):
    from torchpruner_amd.engine.train import native_convs
    model.zero_grad(set_to_none=True)
    torch.manual_seed(123)  # identical dropout masks in both runs
    with native_convs(model, enable=native):
        loss = F.cross_entropy(model(x), y)
        loss.backward()
    return float(loss.detach()), _grads(model)


@pytest.mark.parametrize("arch", ["resnet", "vgg"])
def test_native_conv_training_matches_autograd(cuda, arch):
    from torchpruner_amd import Pruner, get_resnet_pruning_graph, get_vgg_pruning_graph
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    torch.manual_seed(0)
    if arch == "resnet":
        model = ResNet(Bottleneck, [1, 2, 1, 1], num_classes=10, width=32).to(cuda)
        shape, graph = (3, 64, 64), get_resnet_pruning_graph
    else:
        model = prunable_vgg16().to(cuda)
        shape, graph = (3, 32, 32), get_vgg_pruning_graph
        for m in model.modules():  # the native Philox dropout draws other masks than ATen's
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    rng = np.random.RandomState(0)
    pruner = Pruner(model, shape, cuda)
    for module, cascade in graph(model):  # odd widths: channel padding inside the native convs
        n = module.weight.shape[0]
        pruner.prune_model(module, rng.choice(n, int(n * 0.3) + 1, replace=False), cascade)
    model = model.to(memory_format=torch.channels_last).train()
    x = torch.randn(6, *shape, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (6,), device=cuda)
    ref_model = copy.deepcopy(model)
    l_nat, g_nat = _step_grads(model, x, y, True)
    l_ref, g_ref = _step_grads(ref_model, x, y, False)
    assert abs(l_nat - l_ref) < 1e-4 * max(1.0, abs(l_ref))
    for (name, _), a, b in zip(model.named_parameters(), g_nat, g_ref):
        # (conv biases feeding a train-mode BN have ~0 gradient: absolute floor)
        assert (a - b).abs().max().item() <= 2e-3 * b.abs().max().item() + 1e-6, name
    # running statistics were updated identically (BN stays PyTorch)
    for (n1, b1), (_, b2) in zip(model.named_buffers(), ref_model.named_buffers()):
        torch.testing.assert_close(b1.float(), b2.float(), rtol=1e-4, atol=1e-5, msg=n1)


@pytest.mark.parametrize("C,hw,B", [(64, (7, 9), 5), (36, (14, 14), 3), (2048, (2, 2), 4), (4, (33, 1), 2)])
@pytest.mark.parametrize("affine", [True, False])
def test_bn_train_kernels_match_fp64(cuda, C, hw, B, affine):
    """Batch statistics, running-stat update, normalisation and backward vs fp64 F.batch_norm."""
    from torchpruner_amd.engine.train import native_convs
    torch.manual_seed(C + B)
    bn = torch.nn.BatchNorm2d(C, affine=affine).to(cuda).train()
    if affine:
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.5, 0.5)
    ref = copy.deepcopy(bn).double()
    x = (torch.randn(B, C, *hw, device=cuda) * 3 + 1).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(B, C, *hw, device=cuda).contiguous(memory_format=torch.channels_last)
    xr = x.detach().double().requires_grad_(True)
    x = x.requires_grad_(True)
    with native_convs(bn) as sw:
        assert sw == [bn]
        y = bn(x)
    y.backward(gy)
    yr = ref(xr)
    yr.backward(gy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean.double(), ref.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_var.double(), ref.running_var, rtol=1e-5, atol=1e-5)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    if affine:
        torch.testing.assert_close(bn.weight.grad.double(), ref.weight.grad, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(bn.bias.grad.double(), ref.bias.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ks,pad,cin,cout,stride", [(5, 2, 1, 32, 1), (3, 2, 32, 64, 1), (5, 2, 40, 24, 1),
                                                    (3, 1, 3, 64, 1), (3, 0, 36, 32, 1), (5, 1, 4, 8, 1),
                                                    (3, 1, 3, 16, 2)])
def test_native_conv_geometries(cuda, ks, pad, cin, cout, stride):
    """5x5 convs, tiny-Cin (packed 4-channel taps) 3x3 / 5x5 first layers and stride-1 paddings
    other than ks // 2 (FMNIST: conv5x5 p2 on 1 channel, conv3x3 p2; reference
    experiments/models/fmnist.py:12-21): forward, input and weight gradients vs fp64 autograd."""
    from torchpruner_amd.engine.train import eligible, native_convs
    torch.manual_seed(ks * 10 + pad + cin)
    conv = torch.nn.Conv2d(cin, cout, ks, stride=stride, padding=pad).to(cuda)
    assert eligible(conv)
    x = torch.randn(3, cin, 14, 13, device=cuda, requires_grad=True)
    with native_convs(conv):
        y = conv(x)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    c64 = copy.deepcopy(conv).double()
    x64 = x.detach().double().requires_grad_(True)
    y64 = c64(x64)
    (y64 * g.double()).sum().backward()
    torch.testing.assert_close(y.double(), y64, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(conv.weight.grad.double(), c64.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(conv.bias.grad.double(), c64.bias.grad, rtol=1e-4, atol=1e-3)


def test_fmnist_generic_attribution_on_native_convs(cuda):
    """A model the fused engines do not lower (FMNIST conv net) runs the generic hook path with
    its convolutions on the native kernels: Taylor / APoZ scores vs an fp64 CPU oracle."""
    import os
    from torchpruner_amd import APoZAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import FMNISTConvNet
    torch.manual_seed(0)
    model = FMNISTConvNet().to(cuda).eval()
    x = torch.randn(24, 1, 28, 28, device=cuda)
    y = torch.randint(0, 10, (24,), device=cuda)
    mods = [model.conv1, model.conv2, model.fc1]
    m = TaylorAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, cuda)
    got = [m.run(mod) for mod in mods]
    assert m.last_path["path"] == "generic" and m.last_path["native_convs"] == 2, m.last_path
    m64 = copy.deepcopy(model).double().cpu()
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        ref = [TaylorAttributionMetric(m64, DeviceLoader(x.double().cpu(), y.cpu(), 8), F.cross_entropy, "cpu").run(
            mod) for mod in (m64.conv1, m64.conv2, m64.fc1)]
    finally:
        del os.environ["TORCHPRUNER_BACKEND"]
    for a, e in zip(got, ref):
        assert np.abs(a - e).max() / (np.abs(e).max() + 1e-30) < 1e-4
    ap = APoZAttributionMetric(model, DeviceLoader(x, y, 8), F.cross_entropy, cuda).run(model.conv2)
    assert ap.shape == (64,) and np.isfinite(ap).all()


@pytest.mark.parametrize("relu,with_res", [(True, False), (True, True), (False, True), (False, False)])
def test_fused_bn_act_matches_autograd(cuda, relu, with_res):
    """relu?(BN_train(x) + res?) fused (one apply pass; backward masks by the saved output and
    returns the residual gradient) vs PyTorch autograd in fp64: output, running statistics and
    the gradients of x, gamma, beta, res."""
    from torchpruner_amd.engine.train import bn_act
    torch.manual_seed(3)
    bn = torch.nn.BatchNorm2d(36).to(cuda).train()
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.3, 0.3)
    bn64 = copy.deepcopy(bn).double()
    x = torch.randn(4, 36, 9, 7, device=cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    res = torch.randn(4, 36, 9, 7, device=cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True) \
        if with_res else None
    y = bn_act(bn, x, res, relu)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    x64 = x.detach().double().requires_grad_(True)
    r64 = res.detach().double().requires_grad_(True) if with_res else None
    y64 = bn64(x64) + (r64 if with_res else 0)
    if relu:
        y64 = torch.relu(y64)
    (y64 * g.double()).sum().backward()
    torch.testing.assert_close(y.double(), y64, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean.double(), bn64.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), bn64.running_var, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.weight.grad.double(), bn64.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.bias.grad.double(), bn64.bias.grad, rtol=1e-4, atol=1e-4)
    if with_res:
        torch.testing.assert_close(res.grad.double(), r64.grad, rtol=1e-5, atol=1e-6)


def test_native_dropout(cuda):
    """Philox dropout: keep rate ~ 1-p, kept values scaled by 1/(1-p), backward uses the same mask,
    reproducible under torch.manual_seed, NaN inputs stay NaN."""
    from torchpruner_amd.engine.train import native_convs
    drop = torch.nn.Dropout(0.3).train()
    x = torch.randn(1000, 513, device=cuda, requires_grad=True)
    with native_convs(drop):
        torch.manual_seed(5)
        y = drop(x)
        torch.manual_seed(5)
        y2 = drop(x)
    assert torch.equal(y, y2)
    kept = y != 0
    rate = kept.float().mean().item()
    assert abs(rate - 0.7) < 0.01
    torch.testing.assert_close(y[kept], x[kept] / 0.7)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, kept)
    with native_convs(drop):
        z = drop(torch.full((64,), float("nan"), device=cuda))
    assert torch.isnan(z).all()


@pytest.mark.parametrize("cin,cout,hw", [(64, 96, (16, 16)), (40, 32, (10, 14))])
def test_native_conv_winograd_training(cuda, cin, cout, hw):
    """Stride-1 3x3 training convs on the Winograd F(2x2,3x3) kernel (forward and data gradient;
    TUNER.fixed() puts Winograd first) vs fp64 autograd."""
    from torchpruner_amd.engine.fused_chain import TUNER
    from torchpruner_amd.engine.train import native_convs
    torch.manual_seed(cin)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1).to(cuda)
    x = torch.randn(2, cin, *hw, device=cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    with TUNER.fixed(), native_convs(conv):
        y = conv(x)
        g = torch.randn_like(y)
        (y * g).sum().backward()
    c64 = copy.deepcopy(conv).double()
    x64 = x.detach().double().requires_grad_(True)
    (c64(x64) * g.double()).sum().backward()
    torch.testing.assert_close(y.double(), c64(x64), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(conv.weight.grad.double(), c64.weight.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("K,C", [(64, 32), (96, 40)])
def test_wino_weights_kernel(cuda, K, C):
    """GPU Winograd weight transform == fused_chain.winograd_weights (forward and flipped-transposed
    data-gradient operand)."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import winograd_weights
    T = ops.require()
    w = torch.randn(K, C, 3, 3, device=cuda)
    torch.testing.assert_close(T.wino_weights(w, False), winograd_weights(w), rtol=1e-6, atol=1e-7)
    wt = torch.randn(C, K, 3, 3, device=cuda)  # forward weight of a conv with Cout=C, Cin=K
    torch.testing.assert_close(T.wino_weights(wt, True), winograd_weights(wt.flip(2, 3).transpose(0, 1)),
                               rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("B,cin,cout", [(7, 512, 10), (64, 784, 200), (3, 36, 40)])
def test_native_linear_training(cuda, B, cin, cout):
    """nn.Linear on the MFMA GEMM through native_convs: forward, input, weight and bias gradients
    vs fp64 autograd (K4 fwd / dgrad / wgrad)."""
    from torchpruner_amd.engine.train import native_convs
    torch.manual_seed(B + cin)
    lin = torch.nn.Linear(cin, cout).to(cuda)
    x = torch.randn(B, cin, device=cuda, requires_grad=True)
    with native_convs(lin):
        y = lin(x)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    l64 = copy.deepcopy(lin).double()
    x64 = x.detach().double().requires_grad_(True)
    y64 = l64(x64)
    (y64 * g.double()).sum().backward()
    torch.testing.assert_close(y.double(), y64, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lin.weight.grad.double(), l64.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lin.bias.grad.double(), l64.bias.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("O,I,KS,cpad_i,cpad_o", [(64, 32, 3, 32, 64), (40, 36, 3, 64, 64), (64, 3, 7, 4, 64),
                                                   (52, 20, 1, 32, 64), (30, 17, 5, 32, 32)])
def test_pack_conv_weight(cuda, O, I, KS, cpad_i, cpad_o):
    """Weight re-layout kernel == the padded / permuted / flipped torch expressions it replaces."""
    from torchpruner_amd import ops
    T = ops.require()
    w = torch.randn(O, I, KS, KS, device=cuda)
    wp = F.pad(w, (0, 0, 0, 0, 0, cpad_i - I, 0, cpad_o - O))
    kk = -(-KS * KS * cpad_i // 32) * 32
    ref0 = F.pad(wp.permute(0, 2, 3, 1).reshape(cpad_o, -1), (0, kk - KS * KS * cpad_i))
    assert torch.equal(T.pack_conv_weight(w, cpad_o, kk, cpad_i, 0), ref0)
    ref1 = wp.flip(2, 3).permute(1, 2, 3, 0).reshape(cpad_i, -1)
    assert torch.equal(T.pack_conv_weight(w, cpad_i, KS * KS * cpad_o, cpad_o, 1), ref1)
    ref2 = wp.permute(1, 2, 3, 0).reshape(cpad_i, -1)
    assert torch.equal(T.pack_conv_weight(w, cpad_i, KS * KS * cpad_o, cpad_o, 2), ref2)


def test_pack_conv_weights_multi_and_pack_set(cuda):
    """One multi-operand launch == the per-operand pack for contiguous and channels_last weights;
    the training pack cache repacks after an in-place update (version counter) and serves hits
    between updates without a launch."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.train import _PackSet
    T = ops.require()
    shapes = [(64, 32, 3, 32, 64, 0), (40, 36, 3, 64, 64, 1), (64, 3, 7, 4, 64, 0), (52, 20, 1, 32, 64, 2),
              (30, 17, 5, 32, 32, 1)]
    ws, outs, cfg, refs = [], [], [], []
    for i, (O, I, KS, ci, co, mode) in enumerate(shapes):
        w = torch.randn(O, I, KS, KS, device=cuda)
        if i % 2:
            w = w.contiguous(memory_format=torch.channels_last)
        rows, cp = (co, ci) if mode == 0 else (ci, co)
        cols = -(-KS * KS * cp // 32) * 32
        ws.append(w)
        outs.append(torch.full((rows, cols), float("nan"), device=cuda))
        cfg += [rows, cols, cp, mode]
        refs.append(T.pack_conv_weight(w.contiguous(), rows, cols, cp, mode))
    T.pack_conv_weights_multi(ws, outs, cfg)
    for o, r in zip(outs, refs):
        assert torch.equal(o, r)
    ps = _PackSet()
    w = ws[1]
    a = ps.get(T, w, "pack", tuple(cfg[4:8]), tuple(cfg[4:6]))
    assert torch.equal(a, refs[1])
    assert ps.get(T, w, "pack", tuple(cfg[4:8]), tuple(cfg[4:6])) is a  # hit: same buffer, no repack
    with torch.no_grad():
        w.mul_(2.0)  # in-place: version bump -> the next request repacks
    b = ps.get(T, w, "pack", tuple(cfg[4:8]), tuple(cfg[4:6]))
    assert b is a and torch.equal(b, 2.0 * refs[1])


def test_wino4_weights_channels_last(cuda):
    """The F(4x4) weight transform reads a channels_last parameter in place: same U images."""
    from torchpruner_amd import ops
    T = ops.require()
    w = torch.randn(64, 40, 3, 3, device=cuda)
    wl = w.contiguous(memory_format=torch.channels_last)
    assert not wl.is_contiguous()
    for flip in (False, True):
        assert torch.equal(T.wino4_weights(wl, flip, 64, 64), T.wino4_weights(w, flip, 64, 64))
    # the multi-operand launch (training caches): one launch for several weights, both layouts
    w2 = torch.randn(32, 64, 3, 3, device=cuda)
    us = [torch.full((8, 2, T.wino4_u_img()), float("nan"), device=cuda),
          torch.full((8, 2, T.wino4_u_img()), float("nan"), device=cuda),
          torch.full((4, 2, T.wino4_u_img()), float("nan"), device=cuda)]
    T.wino4_weights_multi([wl, w, w2], us, [64, 64, 0, 64, 64, 1, 64, 32, 1])
    assert torch.equal(us[0], T.wino4_weights(w, False, 64, 64))
    assert torch.equal(us[1], T.wino4_weights(w, True, 64, 64))
    assert torch.equal(us[2], T.wino4_weights(w2, True, 64, 32))


@pytest.mark.parametrize("O,I", [(40, 36), (64, 32)])
def test_wino_weights_padded_source(cuda, O, I):
    """Winograd images from an UNPADDED weight == images of the zero-padded weight."""
    from torchpruner_amd import ops
    T = ops.require()
    from torchpruner_amd.engine.fused_chain import cpad
    op, ip = cpad(O), cpad(I)
    w = torch.randn(O, I, 3, 3, device=cuda)
    wp = F.pad(w, (0, 0, 0, 0, 0, ip - I, 0, op - O))
    assert torch.equal(T.wino_weights(w, False, op, ip), T.wino_weights(wp, False))
    assert torch.equal(T.wino_weights(w, True, ip, op), T.wino_weights(wp, True))


@pytest.mark.parametrize("splits", [1, 5])
@pytest.mark.parametrize("channels_last", [False, True])
def test_conv_wgrad_param_layout(cuda, splits, channels_last):
    """conv_wgrad writing the parameter-shaped gradient (real channels, any strides) directly ==
    the sliced / permuted GEMM result."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(splits)
    B, H, W, Cin_p, Cout_p, Cin, Cout, ks = 2, 10, 12, 64, 64, 50, 44, 3
    x = torch.randn(B, H, W, Cin_p, generator=g).to(cuda)
    x[..., Cin:] = 0
    gy = torch.randn(B, H, W, Cout_p, generator=g).to(cuda)
    gy[..., Cout:] = 0
    dwk = T.conv_wgrad(gy, x, ks, 1, 1, 0, splits)
    ref = dwk[:Cout, :ks * ks * Cin_p].view(Cout, ks, ks, Cin_p)[..., :Cin].permute(0, 3, 1, 2)
    out = torch.full((Cout, Cin, ks, ks), float("nan"), device=cuda)
    if channels_last:
        out = out.contiguous(memory_format=torch.channels_last)
    T.conv_wgrad(gy, x, ks, 1, 1, 0, splits, out)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (2, 2, 0), (3, 1, 1), (5, 3, 2)])
def test_native_maxpool_training(cuda, k, s, p):
    """Native max-pool (argmax byte + gather backward) == ATen max_pool2d, incl. ReLU-zero ties and
    NaN propagation (forward value and the gradient's routing)."""
    from torchpruner_amd.engine.train import native_convs
    torch.manual_seed(k * 10 + s)
    x = F.relu(torch.randn(3, 8, 13, 11, device=cuda)).contiguous(memory_format=torch.channels_last)
    x[0, 1, 4, 5] = float("nan")
    mp = torch.nn.MaxPool2d(k, s, p)
    xa = x.detach().clone().requires_grad_(True)
    xb = x.detach().clone().requires_grad_(True)
    with native_convs(mp):
        assert "forward" in mp.__dict__
        ya = mp(xa)
    yb = F.max_pool2d(xb, k, s, p)
    torch.testing.assert_close(ya, yb, equal_nan=True)
    g = torch.randn_like(yb)
    g[torch.isnan(yb)] = 0.0
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-6, atol=1e-6)


def test_native_global_avgpool_training(cuda):
    from torchpruner_amd.engine.train import native_convs
    torch.manual_seed(3)
    x = torch.randn(4, 64, 7, 7, device=cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    gap = torch.nn.AdaptiveAvgPool2d((1, 1))
    with native_convs(gap):
        y = gap(x)
    y2 = F.adaptive_avg_pool2d(x2, 1)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(y2)
    y.backward(g)
    y2.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("B,H,W,Cin,Cout,cin_r,cout_r,splits", [(2, 8, 10, 32, 64, 32, 64, 1), (3, 6, 6, 64, 36, 50, 36, 4),
                                                                (2, 14, 14, 128, 128, 128, 100, 7)])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_wino_wgrad(cuda, B, H, W, Cin, Cout, cin_r, cout_r, splits, cfg):
    """Winograd F(2x2,3x3) weight gradient == fp64 conv2d_weight (stride 1, pad 1), written into a
    parameter-shaped tensor of the real channels."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(B * 100 + Cin + cfg)
    x = torch.randn(B, H, W, Cin, generator=g)
    x[..., cin_r:] = 0
    gy = torch.randn(B, H, W, Cout, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (Cout, Cin, 3, 3),
                                      gy.permute(0, 3, 1, 2).double(), stride=1, padding=1)[:cout_r, :cin_r]
    out = torch.full((cout_r, cin_r, 3, 3), float("nan"), device=cuda)
    T.wino_wgrad(gy.to(cuda), x.to(cuda), cfg, splits, out)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("cfg", [0, 2, 4, 1])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 7, 9, 64, 36), (3, 14, 14, 128, 256)])
def test_conv_gen_stats(cuda, cfg, B, H, W, Cin, Cout):
    """1x1 conv forward with the BN statistics reduced in its epilogue: tile sums fold to the
    fp64 column sums of the output, and bn_train_fwd(pre=) == the statistics-pass forward."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(cfg * 7 + Cin)
    x = torch.randn(B, H, W, Cin, generator=g).to(cuda)
    w = (torch.randn(Cout, Cin, generator=g) * 0.1).to(cuda)
    y, part = T.conv_gen_stats(x, w, None, 1, 1, 0, cfg)
    ref = (x.reshape(-1, Cin).double() @ w.double().t())
    torch.testing.assert_close(y.reshape(-1, Cout).double(), ref, rtol=1e-4, atol=1e-4)
    yd = y.reshape(-1, Cout).double()
    # per-thread fp32 partials over a few rows, folded in fp64: error ~1e-7 of the sum of |terms|
    torch.testing.assert_close(part[:, 0].sum(0), yd.sum(0), rtol=0, atol=1e-6 * float(yd.abs().sum(0).max()))
    torch.testing.assert_close(part[:, 1].sum(0), (yd ** 2).sum(0), rtol=1e-6, atol=1e-6)
    gamma = torch.rand(Cout, device=cuda) + 0.5
    beta = torch.randn(Cout, device=cuda)
    outs = []
    for pre in (None, part):
        rm, rv = torch.zeros(Cout, device=cuda), torch.ones(Cout, device=cuda)
        o = T.bn_train_fwd(y, gamma, beta, rm, rv, 1e-5, 0.1, None, True, pre)
        outs.append((o[0], rm, rv))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kind", ["foreach", "fused"])
def test_pack_cache_follows_optimizer_steps(cuda, kind):
    """The batched weight-pack cache must see every optimizer step: torch's fused SGD updates the
    parameters without bumping their version counters (the post-step hook and the forward epoch
    catch it). Losses with the cache == losses with one pack per call, step by step."""
    from torchpruner_amd.engine import train as tr
    from torchpruner_amd.models import resnet18
    runs = []
    saved = tr._BATCH_PACK
    try:
        for batch_pack in (False, True):
            tr._BATCH_PACK = batch_pack
            torch.manual_seed(0)
            m = resnet18(num_classes=10).to(cuda).to(memory_format=torch.channels_last).train()
            sw = tr.enable_native_convs(m)
            opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, **{kind: True})
            x = torch.randn(8, 3, 32, 32, device=cuda).contiguous(memory_format=torch.channels_last)
            y = torch.randint(0, 10, (8,), device=cuda)
            losses = []
            with tr.TUNER.fixed():
                for _ in range(4):
                    opt.zero_grad(set_to_none=True)
                    loss = F.cross_entropy(m(x), y)
                    loss.backward()
                    opt.step()
                    losses.append(loss.item())
            tr.disable_native_convs(sw)
            runs.append(losses)
    finally:
        tr._BATCH_PACK = saved
    assert runs[0][-1] < runs[0][0]
    for a, b in zip(*runs):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), runs


@pytest.mark.parametrize("B,S,C,N,stride", [(4, 14, 64, 256, 1), (3, 28, 128, 64, 2), (2, 7, 256, 96, 1)])
def test_single_stage_lds_gemm_matches(cuda, B, S, C, N, stride):
    """cfg | CFG_SB (one LDS stage, short-K 1x1 forward) == the double-buffered kernel bit for bit
    (same MFMA order), with and without the BN-statistics epilogue; vs fp64 as well."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import CFG_SB
    T = ops.require()
    torch.manual_seed(0)
    x = torch.randn(B, S, S, C, device=cuda)
    w = torch.randn(N, T.conv_gen_k(1, C), device=cuda) * 0.1
    shift = torch.randn(N, device=cuda)
    ref = torch.einsum("bhwc,nc->bhwn", x[:, ::stride, ::stride].double(), w[:, :C].double()) + shift.double()
    for c in (2, 3, 4, 6):
        y0 = T.conv_gen(x, w, None, shift, False, None, None, 1, stride, 0, c, 1)
        y1 = T.conv_gen(x, w, None, shift, False, None, None, 1, stride, 0, CFG_SB | c, 1)
        assert torch.equal(y0, y1), c
        torch.testing.assert_close(y1.double(), ref, rtol=1e-4, atol=1e-4)
        s0, p0 = T.conv_gen_stats(x, w, shift, 1, stride, 0, c)
        s1, p1 = T.conv_gen_stats(x, w, shift, 1, stride, 0, CFG_SB | c)
        assert torch.equal(s0, s1) and torch.equal(p0, p1), c
        if stride == 1:  # the data gradient with the ReLU mask of the input activation
            g = torch.randn(B, S, S, N, device=cuda)
            wt = w[:, :C].t().contiguous()
            if wt.shape[1] % 32:
                wt = F.pad(wt, (0, 32 - wt.shape[1] % 32))
            gp = F.pad(g, (0, wt.shape[1] - N))
            d0 = T.conv_gen_bwd(gp, wt, None, 1, x, 1, 1, 0, S, S, False, c, 1, None, 0)
            d1 = T.conv_gen_bwd(gp, wt, None, 1, x, 1, 1, 0, S, S, False, CFG_SB | c, 1, None, 0)
            assert torch.equal(d0, d1), c
            dref = torch.einsum("bhwn,nc->bhwc", g.double(), w[:, :C].double()) * (x > 0)
            torch.testing.assert_close(d1.double(), dref, rtol=1e-4, atol=1e-4)
            R = T.conv_gen_tay_slots(c, S * S)
            if R > 0:  # Taylor partials of the activation (the ResNet engine's 1x1 data gradients)
                t0 = torch.zeros(R, B, C, device=cuda)
                t1 = torch.zeros(R, B, C, device=cuda)
                e0 = T.conv_gen_bwd(gp, wt, None, 1, x, 1, 1, 0, S, S, False, c, 1, t0, 0)
                e1 = T.conv_gen_bwd(gp, wt, None, 1, x, 1, 1, 0, S, S, False, CFG_SB | c, 1, t1, 0)
                assert torch.equal(e0, e1) and torch.equal(t0, t1), c
                tref = (-(dref * x.double())).sum((1, 2))
                torch.testing.assert_close(t1.double().sum(0), tref, rtol=1e-3, atol=1e-3)


def test_bottleneck_backward_fusions(cuda):
    """The bottleneck backward fusions (engine/train.py _BNLink): each block tail's BN statistics come
    from the next block's conv1 dgrad epilogue and identity gradients reach conv1's epilogue unmasked
    (masked there by the tail's ReLU bits). Gradients vs fp64 autograd on the same model, and both
    fusions were taken; a second consumer of a block output (a tail hook adding to its gradient) makes
    the tail fall back to its own statistics pass, still exact."""
    from torchpruner_amd.engine import train as tr
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    if not tr._BWD_FUSE:
        pytest.skip("TORCHPRUNER_BN_BWD_FUSE=0")
    torch.manual_seed(3)
    model = ResNet(Bottleneck, [2, 3, 1, 1], num_classes=10, width=16).to(cuda)
    model = model.to(memory_format=torch.channels_last).train()
    x = torch.randn(4, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=cuda)
    m64 = copy.deepcopy(model).double()

    def fp64_grads(extra):
        m64.zero_grad(set_to_none=True)
        feats = {}
        h = m64.layer2[0].register_forward_hook(lambda m, i, o: feats.__setitem__("o", o))
        loss = F.cross_entropy(m64(x.double()), y)
        if extra:
            loss = loss + (feats["o"] ** 2).mean() * 1e-2
        loss.backward()
        h.remove()
        return [p.grad for p in m64.parameters()]

    for extra in (False, True):
        before = dict(tr.FUSE_COUNTS)
        model.zero_grad(set_to_none=True)
        feats = {}
        h = model.layer2[0].register_forward_hook(lambda m, i, o: feats.__setitem__("o", o))
        with tr.native_convs(model):
            loss = F.cross_entropy(model(x), y)
            if extra:  # a second consumer of a block output
                loss = loss + (feats["o"] ** 2).mean() * 1e-2
            loss.backward()
        h.remove()
        got = [p.grad.double() for p in model.parameters()]
        ref = fp64_grads(extra)
        for (name, _), a, b in zip(model.named_parameters(), got, ref):
            assert (a - b).abs().max().item() <= 5e-3 * b.abs().max().item() + 1e-6, (extra, name)
        taken = {k: tr.FUSE_COUNTS[k] - before[k] for k in before}
        assert taken["raw_residual"] >= 3, taken  # identity blocks: 1 + 2 + 0 + 0 ... (+ later layers)
        assert taken["bn_stats_from_dgrad"] >= 4, taken


def test_bottleneck_fusions_release_the_graph(cuda):
    """The _BNLink objects must not keep a finished step's graph alive: pruning in place between two
    steps (new parameter shapes) would then hit the old grad accumulators ("invalid gradient")."""
    from torchpruner_amd import Pruner, get_resnet_pruning_graph
    from torchpruner_amd.engine import train as tr
    from torchpruner_amd.models.resnet import Bottleneck, ResNet
    torch.manual_seed(4)
    model = ResNet(Bottleneck, [2, 2, 1, 1], num_classes=10, width=16).to(cuda)
    model = model.to(memory_format=torch.channels_last).train()
    x = torch.randn(4, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=cuda)
    pruner = Pruner(model, (3, 64, 64), cuda)
    rng = np.random.RandomState(0)
    for step in range(3):
        model.zero_grad(set_to_none=True)
        with tr.native_convs(model):
            loss = F.cross_entropy(model(x), y)
            loss.backward()
        assert torch.isfinite(loss)
        del loss
        for module, cascade in get_resnet_pruning_graph(model):  # every prunable conv, in place
            n = module.weight.shape[0]
            pruner.prune_model(module, rng.choice(n, max(1, n // 8), replace=False), cascade)
        model.train()
