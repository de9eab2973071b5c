"""ResNet residual-aware pruning and prune->finetune under (gloo) DDP with optimizer rewiring."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import APoZAttributionMetric, Pruner, TaylorAttributionMetric, get_resnet_pruning_graph
from torchpruner_amd.data import DeviceLoader
from torchpruner_amd.models import BasicBlock, Bottleneck, ResNet


def tiny_resnet(block=Bottleneck):
    torch.manual_seed(0)
    return ResNet(block, [1, 2, 1, 1], num_classes=10, width=8)


@pytest.mark.parametrize("block", [BasicBlock, Bottleneck])
def test_resnet_pruning_graph_and_prune(block):
    model = tiny_resnet(block).eval()
    graph = get_resnet_pruning_graph(model)
    per_block = 1 if block is BasicBlock else 2
    assert len(graph) == per_block * 5
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    dl = DeviceLoader(x, y, 2)
    pruner = Pruner(model, (3, 32, 32), "cpu")
    for module, cascade in graph:
        s = TaylorAttributionMetric(model, dl, F.cross_entropy, "cpu").run(module, find_best_evaluation_module=True)
        assert s.shape == (module.out_channels,)
        idx = np.argsort(s)[: module.out_channels // 2]
        pruner.prune_model(module, idx, cascade)
    out = model(x)
    assert out.shape == (4, 10) and torch.isfinite(out).all()
    # the residual stream is untouched: block outputs keep their widths
    assert model.fc.in_features == 8 * 8 * block.expansion
    a = APoZAttributionMetric(model, dl, F.cross_entropy, "cpu").run(graph[0][0])
    assert np.isfinite(a).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from torchpruner_amd.parallel import PrunableDDP, params_in_sync
        from torchpruner_amd.utils import train
        model = tiny_resnet()
        g = torch.Generator().manual_seed(5)
        x = torch.randn(16, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (16,), generator=g)
        dl = DeviceLoader(x, y, 4)
        wrapper = PrunableDDP(model)
        opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
        train(wrapper, "cpu", F.cross_entropy, dl, opt, 0, log_every=0)
        pruner = Pruner(model, (3, 32, 32), "cpu", optimizer=opt)
        for module, cascade in get_resnet_pruning_graph(model)[:3]:
            s = TaylorAttributionMetric(model.eval(), dl, F.cross_entropy, "cpu").run(
                module, find_best_evaluation_module=True)
            # rank-dependent garbage indices: the pruner must broadcast rank 0's choice
            idx = np.argsort(s)[:2] if rank == 0 else np.array([module.out_channels - 1])
            pruner.prune_model(module, idx, cascade)
            wrapper.rewrap()
            train(wrapper, "cpu", F.cross_entropy, dl, opt, 1, log_every=0)
        ok = params_in_sync(model)
        if rank == 0:
            torch.save({"ok": ok, "w": [p.detach().clone() for p in model.parameters()]}, path)
    finally:
        dist.destroy_process_group()


def test_prune_finetune_ddp_gloo():
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "out.pt")
        mp.spawn(_worker, args=(2, port, path), nprocs=2, join=True)
        out = torch.load(path, weights_only=False)
    assert out["ok"]
