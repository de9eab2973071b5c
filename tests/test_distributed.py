"""Multi-process data-parallel attribution on the gloo backend (world_size 2, 3, 4, 8; CPU).

Checks that sharded runs reproduce the single-process scores: Taylor/Sensitivity/APoZ with
whole-batch round-robin sharding (R1/R2), Shapley with prefix-work sharding (R3/R4), and
that the pruner broadcasts indices from rank 0 (R5).
"""
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model_and_data():
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import with_forward_partial
    torch.manual_seed(0)
    model = with_forward_partial(nn.Sequential(nn.Conv2d(3, 6, 3, padding=1), nn.BatchNorm2d(6), nn.ReLU(True),
                                               nn.MaxPool2d(2), nn.Conv2d(6, 5, 3, padding=1), nn.ReLU(True),
                                               nn.Flatten(), nn.Linear(5 * 16, 4))).eval()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(22, 3, 8, 8, generator=g)
    y = torch.randint(0, 4, (22,), generator=g)
    return model, DeviceLoader(x, y, 4)  # 6 batches, last one ragged


def _compute(world_rank=None):
    from torchpruner_amd import (APoZAttributionMetric, Pruner, SensitivityAttributionMetric,
                                 ShapleyAttributionMetric, TaylorAttributionMetric)
    model, dl = _model_and_data()
    dev = torch.device("cpu")
    out = {}
    out["taylor"] = TaylorAttributionMetric(model, dl, F.cross_entropy, dev).run(model[0], find_best_evaluation_module=True)
    out["taylor_none"] = TaylorAttributionMetric(model, dl, F.cross_entropy, dev, reduction="none").run(model[4])
    out["sens_sum"] = SensitivityAttributionMetric(model, dl, F.cross_entropy, dev, reduction="sum").run(model[4])
    out["apoz_many"] = APoZAttributionMetric(model, dl, F.cross_entropy, dev).run_many([model[0], model[4]], True)
    np.random.seed(7)
    out["sv"] = ShapleyAttributionMetric(model, dl, F.cross_entropy, dev, sv_samples=3, prefix_batch=2).run(model[4])
    np.random.seed(7)
    out["sv_none"] = ShapleyAttributionMetric(model, dl, F.cross_entropy, dev, sv_samples=2,
                                              reduction="none").run(model[0], find_best_evaluation_module=True)
    # a per-rank ShardLoader with fewer batches (2) than ranks: sharded by batches
    from torchpruner_amd.data import ShardLoader
    world = dist.get_world_size() if dist.is_initialized() else 1
    rk = dist.get_rank() if dist.is_initialized() else 0
    xs, ys = next(iter(dl))
    sl = ShardLoader.build(lambda i: (xs + i, ys), 2, xs.shape[0], rk, world)
    np.random.seed(5)
    out["sv_shard"] = ShapleyAttributionMetric(model, sl, F.cross_entropy, dev, sv_samples=2).run(model[4])
    # pruner: rank-dependent indices must be replaced by rank 0's
    rank = dist.get_rank() if dist.is_initialized() else 0
    Pruner(model, (3, 8, 8), dev).prune_model(model[4], [rank, 3], [model[7]])
    out["pruned_w"] = model[4].weight.detach().numpy().copy()
    return out


def _worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        out = _compute()
        if rank == 0:
            torch.save({k: v for k, v in out.items()}, path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_dp_matches_single_process(world):
    ref = _compute()
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "out.pt")
        mp.spawn(_worker, args=(world, port, path), nprocs=world, join=True)
        got = torch.load(path, weights_only=False)
    # fp64 device accumulators: the sharded reductions agree with one process to <= 1e-6
    # relative; Shapley work is cut on the single-rank prefix-chunk grid and its
    # deltas summed unscaled, so it is bit-identical (world 8: 6 batches -> prefix split)
    for k in ["taylor", "taylor_none", "sens_sum"]:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-6, atol=1e-9, err_msg=k)
    for k in ["sv", "sv_none", "sv_shard"]:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for a, b in zip(got["apoz_many"], ref["apoz_many"]):
        np.testing.assert_allclose(a, b, rtol=1e-6)
    assert got["taylor_none"].shape == (22, 5)
    np.testing.assert_array_equal(got["pruned_w"], ref["pruned_w"])  # rank 0 indices [0, 3] everywhere


def test_repeat_runs_bit_identical():
    """Same seed, same world size -> bit-identical scores (no atomics on the CPU paths)."""
    a, b = _compute(), _compute()
    for k in a:
        if isinstance(a[k], list):
            for x, y in zip(a[k], b[k]):
                np.testing.assert_array_equal(x, y, err_msg=k)
        else:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
