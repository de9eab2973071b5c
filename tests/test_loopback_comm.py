"""Data-parallel attribution through the in-process loopback Communicator.

N ranks run as N threads of this process (no sockets, no process spawn); every metric gets
``group=<LoopbackCommunicator>``. The sharded results must equal the single-process ones, as in
the gloo multi-process tests (tests/test_distributed.py), and repeated loopback runs must be
bit-identical (reductions are summed in rank order).
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import (APoZAttributionMetric, Pruner, SensitivityAttributionMetric, ShapleyAttributionMetric,
                             TaylorAttributionMetric)
from torchpruner_amd.data import DeviceLoader
from torchpruner_amd.models import with_forward_partial
from torchpruner_amd.parallel import LoopbackCommunicator, LoopbackHub, get_rank, get_world_size, run_loopback
from torchpruner_amd.parallel import dist as pdist
from torchpruner_amd.parallel.ddp import params_in_sync


def _model_and_data():
    torch.manual_seed(0)
    model = with_forward_partial(nn.Sequential(nn.Conv2d(3, 6, 3, padding=1), nn.BatchNorm2d(6), nn.ReLU(True),
                                               nn.MaxPool2d(2), nn.Conv2d(6, 5, 3, padding=1), nn.ReLU(True),
                                               nn.Flatten(), nn.Linear(5 * 16, 4))).eval()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(22, 3, 8, 8, generator=g)
    y = torch.randint(0, 4, (22,), generator=g)
    return model, x, y


def _compute(model, x, y, comm=None):
    dev = torch.device("cpu")
    dl = DeviceLoader(x, y, 4)  # 6 batches, the last one ragged
    rank = 0 if comm is None else comm.rank
    out = {}
    out["taylor"] = TaylorAttributionMetric(model, dl, F.cross_entropy, dev, group=comm).run(
        model[0], find_best_evaluation_module=True)
    out["taylor_none"] = TaylorAttributionMetric(model, dl, F.cross_entropy, dev, reduction="none",
                                                 group=comm).run(model[4])
    out["sens_sum"] = SensitivityAttributionMetric(model, dl, F.cross_entropy, dev, reduction="sum",
                                                   group=comm).run(model[4])
    out["apoz_many"] = APoZAttributionMetric(model, dl, F.cross_entropy, dev, group=comm).run_many(
        [model[0], model[4]], True)
    if rank == 0:  # only rank 0 draws the permutations (broadcast, R3)
        np.random.seed(7)
    out["sv"] = ShapleyAttributionMetric(model, dl, F.cross_entropy, dev, sv_samples=3, prefix_batch=2,
                                         group=comm).run(model[4])
    # pruner: rank-dependent indices are replaced by rank 0's (R5)
    Pruner(model, (3, 8, 8), dev, group=comm).prune_model(model[4], [rank, 3], [model[7]])
    out["pruned_w"] = model[4].weight.detach().numpy().copy()
    out["in_sync"] = params_in_sync(model, comm)
    return out


def _loopback(world):
    model, x, y = _model_and_data()
    models = [copy.deepcopy(model) for _ in range(world)]
    return run_loopback(world, lambda comm: _compute(models[comm.rank], x, y, comm))


def _close(a, b):
    if isinstance(a, list):
        return all(_close(u, v) for u, v in zip(a, b))
    if isinstance(a, (bool, np.bool_)):
        return a == b
    return a.shape == b.shape and np.allclose(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_loopback_dp_matches_single_process(world):
    model, x, y = _model_and_data()
    ref = _compute(model, x, y)
    outs = _loopback(world)
    for r, out in enumerate(outs):
        for k, v in ref.items():
            assert _close(v, out[k]), (world, r, k)


def test_loopback_bit_identical_repeat():
    a, b = _loopback(3), _loopback(3)
    for k in a[0]:
        if k == "in_sync":
            continue
        got, want = a[0][k], b[0][k]
        if isinstance(got, list):
            assert all(np.array_equal(u, v) for u, v in zip(got, want)), k
        else:
            assert np.array_equal(got, want), k


def test_loopback_collectives():
    def body(comm):
        t = torch.full((3,), float(comm.rank + 1))
        pdist.all_reduce_sum_(t, comm)
        b = torch.full((2,), float(comm.rank))
        pdist.broadcast_tensor_(b, 1, comm)
        rows = pdist.gather_ordered_rows([(comm.rank + 10 * i, torch.full((i + 1, 2), float(comm.rank)))
                                          for i in range(2)], comm)
        pdist.barrier(comm)
        return (get_rank(comm), get_world_size(comm), t.tolist(), b.tolist(), rows[:, 0].tolist(),
                pdist.all_max_int(comm.rank * 5, comm), pdist.all_max_float(-comm.rank, comm),
                pdist.broadcast_object({"r": comm.rank}, 2, comm))

    outs = run_loopback(3, body)
    for r, (rank, world, t, b, rows, mi, mf, obj) in enumerate(outs):
        assert (rank, world) == (r, 3)
        assert t == [6.0] * 3 and b == [1.0, 1.0]
        # global batch order: indices 0,1,2 (one row each) then 10,11,12 (two rows each)
        assert rows == [0.0, 1.0, 2.0, 0.0, 0.0, 1.0, 1.0, 2.0, 2.0]
        assert mi == 10 and mf == 0.0 and obj == {"r": 2}


def test_loopback_error_propagates_without_hang():
    def body(comm):
        if comm.rank == 1:
            raise ValueError("rank 1 failed")
        comm.barrier()

    with pytest.raises(ValueError, match="rank 1 failed"):
        run_loopback(2, body)


def test_communicator_single_rank_is_identity():
    hub = LoopbackHub(1)
    comm = LoopbackCommunicator(hub, 0)
    t = torch.arange(4.0)
    assert pdist.all_reduce_sum_(t, comm) is t and t.tolist() == [0.0, 1.0, 2.0, 3.0]
    assert get_world_size(comm) == 1 and get_rank(comm) == 0


def test_loopback_mismatched_collectives_raise():
    """A rank calling broadcast_ while another calls all_reduce_ must fail, not mix payloads."""
    def body(comm):
        t = torch.ones(3)
        if comm.rank == 0:
            comm.broadcast_(t, 0)
        else:
            comm.all_reduce_(t)

    with pytest.raises(RuntimeError, match="mismatched collectives"):
        run_loopback(2, body)


def test_loopback_all_gather_outputs_are_private():
    def body(comm):
        outs = comm.all_gather(torch.full((2,), float(comm.rank)))
        comm.barrier()
        if comm.rank == 0:
            for o in outs:
                o.fill_(-1.0)  # must not reach rank 1's results
        comm.barrier()
        return [o.tolist() for o in outs]

    res = run_loopback(2, body)
    assert res[1] == [[0.0, 0.0], [1.0, 1.0]]


def test_shapley_work_split_modes():
    """Shapley shards whole batches when every rank gets one (no replicated upstream forward),
    else splits each batch's prefixes across ranks."""
    model, x, y = _model_and_data()
    dl = DeviceLoader(x, y, 4)  # 6 batches

    def body(comm):
        m = ShapleyAttributionMetric(model, dl, F.cross_entropy, torch.device("cpu"), group=comm)
        return m._work_split()

    assert run_loopback(3, body) == ["batches"] * 3
    assert run_loopback(4, body) == ["hybrid"] * 4  # 6 = 4 whole + 2 prefix-split
    assert run_loopback(8, body) == ["prefixes"] * 8
    assert ShapleyAttributionMetric(model, dl, F.cross_entropy, torch.device("cpu"))._work_split() is None


def test_pruner_lower_level_api_syncs_indices():
    """R5 at every API level: prune_module / prune_parameter called with rank-local indices
    prune rank 0's indices on every replica (one broadcast at the outermost call)."""
    import torch.nn as nn

    w0 = torch.arange(24, dtype=torch.float32).view(6, 4)

    def body(comm):  # (threads share the global RNG: deterministic weights instead of a seed)
        lin = nn.Linear(4, 6)
        lin.weight.data.copy_(w0)
        bn = nn.BatchNorm1d(6)
        p = Pruner(nn.Sequential(lin, bn), (4,), "cpu", group=comm)
        p.prune_module(lin, [comm.rank, 5], direction="out")  # rank-local indices
        p.prune_parameters(bn, ["weight", "bias", "running_mean", "running_var"], [comm.rank + 1])
        p.prune_parameter(lin, "weight", [comm.rank], axis=1)
        return lin.weight.detach().clone(), bn.weight.shape[0]

    outs = run_loopback(3, body)
    for w, nbn in outs:
        assert torch.equal(w, outs[0][0]) and w.shape == (4, 3) and nbn == 5
    # rank 0's choices: out rows {0, 5} removed, then input column 0
    ref = w0[[1, 2, 3, 4]][:, [1, 2, 3]]
    assert torch.equal(outs[0][0], ref)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("reduction", ["mean", "none"])
def test_shapley_balanced_sharding_bit_exact(world, reduction):
    """10 batches on 8 ranks: whole batches for the first 8, the last 2
    prefix-split on the single-rank chunk grid. Scores are bit-identical to one rank at every
    world size, and the prefix work per rank is balanced (max / mean <= 1.1). The losses span a
    wide range (a few near-zero, most large) to exercise the fp64 sums of fp32 deltas."""
    torch.manual_seed(0)
    model = with_forward_partial(nn.Sequential(nn.Linear(6, 48), nn.ReLU(), nn.Linear(48, 4))).eval()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(40, 6, generator=g) * torch.logspace(-3, 2, 40).view(40, 1)
    y = torch.randint(0, 4, (40,), generator=g)
    dl = DeviceLoader(x, y, 4)  # 10 batches

    def body(comm):
        if comm is None or comm.rank == 0:
            np.random.seed(9)
        m = ShapleyAttributionMetric(model, dl, F.cross_entropy, torch.device("cpu"), sv_samples=3, prefix_batch=3,
                                     reduction=reduction, group=comm)
        return m.run(model[0]), m.last_work, m._work_split()

    ref, ref_work, _ = body(None)
    outs = run_loopback(world, body) if world > 1 else [body(None)]
    for sv, _, split in outs:
        np.testing.assert_array_equal(sv, ref)
        if world == 8:
            assert split == "hybrid"
    evals = np.array([w["prefix_evals"] for _, w, _ in outs], dtype=float)
    if world > 1:
        assert evals.max() / evals.mean() <= 1.1, evals
        # nothing but the boundary evaluations of the split ranges is redone
        assert evals.sum() <= ref_work["prefix_evals"] * 1.25, (evals.sum(), ref_work)
