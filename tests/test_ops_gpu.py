"""HIP kernel numerics vs the plain-PyTorch fp32 reference of the same op (CPU oracle)."""
import pytest
import torch

from torchpruner_amd import ops

pytestmark = pytest.mark.gpu

SHAPES = [(4, 64, 32, 32), (8, 128, 16, 16), (16, 512, 4, 4), (32, 512, 2, 2), (8, 512), (3, 7, 5, 3), (2, 3, 1, 1),
          (2, 64, 112, 112), (3, 80, 56, 56), (2, 96, 7, 7), (5, 1056, 3, 3), (256, 32, 9, 9)]


def _ref(fn, *ts):
    import os
    old = os.environ.get("TORCHPRUNER_BACKEND")
    os.environ["TORCHPRUNER_BACKEND"] = "torch"
    try:
        return fn(*[t.cpu() if isinstance(t, torch.Tensor) else t for t in ts])
    finally:
        if old is None:
            del os.environ["TORCHPRUNER_BACKEND"]
        else:
            os.environ["TORCHPRUNER_BACKEND"] = old


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["taylor", "taylor_signed", "sensitivity", "apoz", "sum_grad"])
@pytest.mark.parametrize("cl", [False, True])
def test_channel_reduce(cuda, shape, mode, cl):
    if cl and len(shape) != 4:
        pytest.skip("channels_last needs 4D")
    g = torch.Generator().manual_seed(0)
    a = torch.randn(shape, generator=g)
    gr = torch.randn(shape, generator=g)
    ref = _ref(lambda x, y: ops.channel_reduce(x, y, mode), a, gr)
    ad, gd = a.to(cuda), gr.to(cuda)
    if cl:
        ad = ad.contiguous(memory_format=torch.channels_last)
        gd = gd.contiguous(memory_format=torch.channels_last)
    out = ops.channel_reduce(ad, gd, mode)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-4)


def test_column_accumulate(cuda):
    v = torch.randn(1000, 300)
    s = torch.zeros(300, dtype=torch.float64, device=cuda)
    q = torch.zeros(300, dtype=torch.float64, device=cuda)
    ops.column_accumulate(v.to(cuda), s, q)
    ops.column_accumulate(v.to(cuda), s, q)
    torch.testing.assert_close(s.cpu(), 2 * v.double().sum(0))
    torch.testing.assert_close(q.cpu(), 2 * (v.double() ** 2).sum(0))


def test_fill_and_nan(cuda):
    x = torch.randn(2, 6, 3, 3, device=cuda)
    ops.channel_fill_(x, [1, 4], float("nan"))
    m = ops.nan_channels(x)
    assert m.cpu().tolist() == [False, True, False, False, True, False]
    ops.channel_fill_(x, [1, 4], 0.0)
    assert not ops.nan_channels(x).any()
    assert (x[:, 1] == 0).all() and (x[:, 4] == 0).all()


def test_gather_multi(cuda):
    ts = [torch.randn(8, 5, 3, 3), torch.randn(8), torch.randn(4, 8).double(), torch.randn(8, 2).half()]
    axes = [0, 0, 1, 0]
    keep = torch.tensor([0, 2, 3, 7])
    outs = ops.gather_multi([t.to(cuda) for t in ts], axes, keep.to(cuda))
    for t, ax, o in zip(ts, axes, outs):
        torch.testing.assert_close(o.cpu(), t.index_select(ax, keep))


@pytest.mark.parametrize("cl", [False, True])
def test_prefix_mask(cuda, cl):
    z = torch.randn(3, 8, 4, 4)
    perm = torch.randperm(8)
    rank = torch.empty(8, dtype=torch.int32)
    rank[perm] = torch.arange(8, dtype=torch.int32)
    ref = _ref(lambda a, r: ops.prefix_mask(a, r, 2, 4), z, rank)
    zd = z.to(cuda)
    if cl:
        zd = zd.contiguous(memory_format=torch.channels_last)
    out = ops.prefix_mask(zd, rank.to(cuda), 2, 4)
    torch.testing.assert_close(out.cpu(), ref)


def test_shapley_scatter_column(cuda):
    L = torch.randn(6, 10)
    perm = torch.randperm(12).int()
    sv = torch.zeros(20, 12, dtype=torch.float64)
    _ref(lambda a, p, s: ops.shapley_scatter(a, p, s, 3, 4, 0.2), L, perm, sv)
    svd = torch.zeros(20, 12, dtype=torch.float64, device=cuda)
    ops.shapley_scatter(L.to(cuda), perm.to(cuda), svd, 3, 4, 0.2)
    torch.testing.assert_close(svd.cpu(), sv)
    col = torch.zeros(12, dtype=torch.float64)
    _ref(lambda a, p, s: ops.shapley_column(a, p, s, 4, 0.2), L, perm, col)
    cold = torch.zeros(12, dtype=torch.float64, device=cuda)
    ops.shapley_column(L.to(cuda), perm.to(cuda), cold, 4, 0.2)
    torch.testing.assert_close(cold.cpu(), col)


@pytest.mark.parametrize("nc", [10, 1000])
def test_cross_entropy(cuda, nc):
    x = torch.randn(37, nc) * 3
    t = torch.randint(0, nc, (37,))
    l_ref, g_ref = _ref(lambda a, b: ops.cross_entropy(a, b, 1 / 37, True), x, t)
    l, g = ops.cross_entropy(x.to(cuda), t.to(cuda), 1 / 37, True)
    torch.testing.assert_close(l.cpu(), l_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(g.cpu(), g_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("after", [0, 1, 2])
@pytest.mark.parametrize("take_abs", [False, True])
def test_score_fold_slots(cuda, after, take_abs):
    """(R, B, C) partial slots: summed in slot order, then |.|, fp64 accumulate, keep/zero."""
    g = torch.Generator().manual_seed(10 + after)
    Ts = [torch.randn(r, 9, c, generator=g) for r, c in ((1, 5), (4, 64), (3, 130))] + [torch.randn(6, 33,
                                                                                                  generator=g)]
    cpu = [t.clone() for t in Ts]
    acc_cpu = [torch.zeros(t.shape[-1], dtype=torch.float64) for t in Ts]
    ops.score_fold_(cpu, acc_cpu, take_abs, after)  # PyTorch reference (CPU tensors)
    Td = [t.to(cuda) for t in Ts]
    accs = [torch.zeros(t.shape[-1], dtype=torch.float64, device=cuda) for t in Ts]
    ops.score_fold_(Td, accs, take_abs, after)
    for t, r, a, ar in zip(Td, cpu, accs, acc_cpu):
        torch.testing.assert_close(a.cpu(), ar)
        torch.testing.assert_close(t.cpu(), r)


@pytest.mark.parametrize("after", [0, 1, 2])
@pytest.mark.parametrize("take_abs", [False, True])
def test_score_fold(cuda, after, take_abs):
    g = torch.Generator().manual_seed(after)
    Ts = [torch.randn(7, c, generator=g) for c in (3, 64, 130, 512)] * 5  # 20 slabs -> 2 launches
    ref_T = [t.abs() if take_abs else t.clone() for t in Ts]
    acc_ref = [torch.full((t.shape[1],), 0.5, dtype=torch.float64) + r.double().sum(0) for t, r in zip(Ts, ref_T)]
    Td = [t.to(cuda) for t in Ts]
    accs = [torch.full((t.shape[1],), 0.5, dtype=torch.float64, device=cuda) for t in Ts]
    accs[3] = None
    ops.score_fold_(Td, accs, take_abs, after)
    for i, (t, a) in enumerate(zip(Td, accs)):
        if a is not None:
            torch.testing.assert_close(a.cpu(), acc_ref[i])
        exp = Ts[i] if after == 0 else (ref_T[i] if after == 1 else torch.zeros_like(Ts[i]))
        torch.testing.assert_close(t.cpu(), exp)
