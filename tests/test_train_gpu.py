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
