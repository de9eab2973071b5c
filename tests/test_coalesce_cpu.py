"""The batch-coalescing generator of the fused engine passes (attributions/base.py
_coalesced_batches), on CPU tensors with the factor forced: runs of k equal-shape batches come
concatenated with their loader batch size as ``loss_batch`` and the group's first global index;
a batch of another shape flushes the pending group one batch at a time; leftovers run alone."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchpruner_amd import TaylorAttributionMetric


def _metric(sizes, k):
    data = [(torch.full((s, 3), float(i)), torch.full((s,), i, dtype=torch.long)) for i, s in enumerate(sizes)]
    m = TaylorAttributionMetric(nn.Sequential(nn.Linear(3, 2)), data, F.cross_entropy, "cpu")
    m._coalesce_factor = lambda x: k
    return m


def test_groups_leftovers_and_odd_shapes():
    m = _metric([4, 4, 4, 4, 4, 4, 4, 2], k=3)
    out = list(m._coalesced_batches(True))
    assert [(i, x.shape[0], lb) for i, x, _, lb in out] == [(0, 12, 4), (3, 12, 4), (6, 4, None), (7, 2, None)]
    i, x, y, lb = out[1]
    assert torch.equal(x[:, 0], torch.tensor([3.0] * 4 + [4.0] * 4 + [5.0] * 4))  # batches 3, 4, 5 in order
    assert torch.equal(y, torch.tensor([3] * 4 + [4] * 4 + [5] * 4))
    assert m.last_coalesce == 3


def test_off_and_factor_one_pass_batches_through():
    for on, k in ((False, 3), (True, 1)):
        m = _metric([4, 4, 4], k=k)
        out = list(m._coalesced_batches(on))
        assert [(i, x.shape[0], lb) for i, x, _, lb in out] == [(0, 4, None), (1, 4, None), (2, 4, None)]
        assert m.last_coalesce == 1


def test_shape_change_mid_group_flushes_in_order():
    m = _metric([4, 4, 6, 6, 6], k=3)
    out = list(m._coalesced_batches(True))
    assert [(i, x.shape[0], lb) for i, x, _, lb in out] == [(0, 4, None), (1, 4, None), (2, 18, 6)]


def test_factor_from_env(monkeypatch):
    class _X:  # stands for a CUDA batch (the factor is 1 for CPU tensors)
        is_cuda, shape = True, (100, 3, 32, 32)

    m = _metric([4], k=1)
    del m._coalesce_factor  # the method, not the instance override
    for env, want in (("0", 1), ("1", (3 << 19) // (100 * 3 * 32 * 32)), ("7", 7)):
        monkeypatch.setenv("TORCHPRUNER_COALESCE", env)
        assert m._coalesce_factor(_X()) == want, env
