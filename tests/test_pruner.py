"""Golden parity with the reference pruner suite (torchpruner/tests/test_pruner.py), on CPU and
(marked ``gpu``) MI355X, plus the deliberate fixes (Adam states, metadata, Dropout2d, ...)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from torchpruner.pruner import Pruner

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        from torchpruner_amd import ops
        ops.require()
    return torch.device(name)


def simple_model(device):
    x, y = torch.ones((10, 3)), torch.randint(0, 10, (10, 1))
    return (x.to(device), y.to(device)), nn.Sequential(nn.Linear(3, 2), nn.ReLU(), nn.Linear(2, 1)).to(device)


@pytest.mark.parametrize("dev", DEVICES)
def test_prune_parameter(dev):
    d = _dev(dev)
    (x, y), model = simple_model(d)
    p = Pruner(model, input_size=(3,), device=d)
    module = list(model.children())[0]
    weight_id = id(module.weight)
    p.prune_parameter(module, "weight", [0], axis=0)
    p.prune_parameter(module, "bias", [0], axis=0)
    assert list(module.weight.data.shape) == [1, 3]
    assert list(module.bias.data.shape) == [1]
    assert id(module.weight) == weight_id
    p.prune_parameter(module, "weight", [0], axis=1)
    assert list(module.weight.data.shape) == [1, 2]


@pytest.mark.parametrize("dev", DEVICES)
def test_prune_module_linear(dev):
    d = _dev(dev)
    (x, y), model = simple_model(d)
    p = Pruner(model, input_size=(3,), device=d)
    module = list(model.children())[0]
    p.prune_module(module, [0], direction="out")
    assert list(module.weight.data.shape) == [1, 3]
    assert module.out_features == 1
    p.prune_module(module, [0], direction="in")
    assert list(module.weight.data.shape) == [1, 2]
    assert module.in_features == 2


def _probe(model, input_size, src, dst_list, d, indices=(0,)):
    p = Pruner(model, input_size=input_size, device=d)
    hs = [src.register_forward_hook(p._nanify_hook(list(indices)))]
    hs += [m.register_forward_hook(p._detect_nan_hook()) for m in dst_list]
    p._run_forward()
    for h in hs:
        h.remove()
    return [list(getattr(m, "_nan_indices")) for m in dst_list]


@pytest.mark.parametrize("dev", DEVICES)
def test_nan_trick_linear_linear(dev):
    d = _dev(dev)
    model = nn.Sequential(nn.Linear(3, 2), nn.ReLU(), nn.Linear(2, 1)).to(d)
    assert _probe(model, (3,), model[0], [model[2]], d) == [[0]]


@pytest.mark.parametrize("dev", DEVICES)
def test_nan_trick_conv2d_linear(dev):
    d = _dev(dev)
    model = nn.Sequential(nn.Conv2d(1, 3, 2), nn.ReLU(), nn.Flatten(), nn.Linear(12, 1)).to(d)
    assert _probe(model, (1, 3, 3), model[0], [model[3]], d) == [[0, 1, 2, 3]]


@pytest.mark.parametrize("dev", DEVICES)
def test_nan_trick_conv2d_max_linear(dev):
    d = _dev(dev)
    model = nn.Sequential(nn.Conv2d(1, 3, 2), nn.ReLU(), nn.MaxPool2d(2), nn.Flatten(), nn.Linear(3, 1)).to(d)
    assert _probe(model, (1, 3, 3), model[0], [model[4]], d) == [[0]]


@pytest.mark.parametrize("dev", DEVICES)
def test_nan_trick_linear_bn_linear(dev):
    d = _dev(dev)
    model = nn.Sequential(nn.Linear(3, 2), nn.BatchNorm1d(2), nn.Linear(2, 1)).to(d)
    assert _probe(model, (3,), model[0], [model[1], model[2]], d) == [[0], [0]]


@pytest.mark.parametrize("dev", DEVICES)
def test_prune_model_linear(dev):
    d = _dev(dev)
    (x, y), model = simple_model(d)
    p = Pruner(model, input_size=(3,), device=d)
    module, next_module = list(model.children())[0], list(model.children())[2]
    p.prune_model(module, [0], cascading_modules=[next_module])
    assert list(module.weight.data.shape) == [1, 3]
    assert list(next_module.weight.data.shape) == [1, 1]
    assert list(model(x).shape) == list(y.shape)
    assert not hasattr(next_module, "_nan_indices") and not hasattr(next_module, "_activation_len")


@pytest.mark.parametrize("dev", DEVICES)
def test_prune_model_linear_bn(dev):
    d = _dev(dev)
    (x, y), _ = simple_model(d)
    model = nn.Sequential(nn.Linear(3, 2), nn.BatchNorm1d(2), nn.Linear(2, 1)).to(d)
    rm_before = model[1].running_mean.clone()
    p = Pruner(model, input_size=(3,), device=d)
    module, bn_module, lin_module = model[0], model[1], model[2]
    p.prune_model(module, [0], [bn_module, lin_module])
    assert list(module.weight.data.shape) == [1, 3]
    assert list(lin_module.weight.data.shape) == [1, 1]
    for t in (bn_module.weight, bn_module.bias, bn_module.running_var, bn_module.running_mean):
        assert list(t.data.shape) == [1]
    assert bn_module.num_features == 1
    # the probe must not have touched the running stats of the surviving channel
    assert torch.equal(bn_module.running_mean.cpu(), rm_before[1:].cpu())
    assert list(model(x).shape) == list(y.shape)


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("drop", [nn.Dropout, nn.Dropout1d])
def test_prune_model_linear_dropout(dev, drop):
    d = _dev(dev)
    model = nn.Sequential(nn.Linear(3, 5), drop(0.5), nn.Linear(5, 1)).to(d)
    p = Pruner(model, input_size=(3,), device=d)
    assert model[1].p == 0.5
    p.prune_model(model[0], [0], [model[1], model[2]])
    assert model[1].p == pytest.approx(0.5 * 4 / 5)


def _step(model, x, opt):
    opt.zero_grad()
    model(x).mean().backward()
    opt.step()


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("opt_name", ["sgd", "sgd_momentum", "adam"])
def test_prune_model_with_optimizer(dev, opt_name):
    d = _dev(dev)
    (x, y), _ = simple_model(d)
    model = nn.Sequential(nn.Linear(3, 2), nn.BatchNorm1d(2), nn.Linear(2, 1)).to(d)
    if opt_name == "sgd":
        opt = torch.optim.SGD(model.parameters(), lr=0.01)
    elif opt_name == "sgd_momentum":
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.01)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=0.01)
    p = Pruner(model, input_size=(3,), device=d, optimizer=opt)
    _step(model, x, opt)
    if opt_name != "sgd":
        key = "momentum_buffer" if opt_name == "sgd_momentum" else "exp_avg"
        before = opt.state[model[0].weight][key].clone()
    p.prune_model(model[0], [0], [model[1], model[2]])
    if opt_name != "sgd":
        after = opt.state[model[0].weight][key]
        assert after.shape == model[0].weight.shape
        torch.testing.assert_close(after, before[1:])
        assert opt.state[model[2].weight][key].shape == model[2].weight.shape
    _step(model, x, opt)  # must not raise after pruning


@pytest.mark.parametrize("dev", DEVICES)
def test_prune_conv_chain_with_grads(dev):
    """Conv -> BN -> ReLU -> MaxPool -> Conv -> Flatten -> Linear cascade with live .grad."""
    d = _dev(dev)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(True), nn.MaxPool2d(2),
                          nn.Conv2d(8, 6, 3, padding=1), nn.ReLU(True), nn.Flatten(), nn.Linear(6 * 16, 4)).to(d)
    x = torch.randn(4, 3, 8, 8, device=d)
    model(x).sum().backward()
    p = Pruner(model, input_size=(3, 8, 8), device=d)
    p.prune_model(model[0], [1, 5, 6], [model[1], model[4]])
    assert model[0].weight.shape == (5, 3, 3, 3) and model[0].weight.grad.shape == (5, 3, 3, 3)
    assert model[4].weight.shape == (6, 5, 3, 3) and model[4].in_channels == 5
    p.prune_model(model[4], [0, 2], [model[7]])
    assert model[7].weight.shape == (4, 4 * 16)
    assert model(x).shape == (4, 4)


@pytest.mark.parametrize("dev", DEVICES)
def test_grouped_conv_rejected(dev):
    d = _dev(dev)
    model = nn.Sequential(nn.Conv2d(4, 4, 3, groups=2), nn.Conv2d(4, 2, 1)).to(d)
    p = Pruner(model, input_size=(4, 5, 5), device=d)
    with pytest.raises(NotImplementedError):
        p.prune_module(model[0], [0], "out")


@pytest.mark.parametrize("dev", DEVICES)
def test_out_of_range_indices_raise(dev):
    """Reference parity (pruner.py:106-107 raises through numpy): an index >= the axis length is
    an error, not silently dropped."""
    d = _dev(dev)
    _, model = simple_model(d)
    pruner = Pruner(model, (3,), d)
    with pytest.raises(IndexError):
        pruner.prune_parameter(model[0], "weight", [0, 5], axis=0)
    assert model[0].weight.shape == (2, 3)  # untouched
    with pytest.raises(IndexError):
        pruner.prune_model(model[0], [2], cascading_modules=[model[2]])
