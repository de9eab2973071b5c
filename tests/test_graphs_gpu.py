"""HIP-graph replay of the fused engine's Taylor step (small, launch-bound batches).

The graphed path must give bit-identical scores to the eager launches (the engine's kernels are
deterministic), survive ragged last batches (own graph per shape), and notice re-packed weights
(pruning / BN changes invalidate the captured graph)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _scores(model, x, y, B, env, **kw):
    from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    metric = SensitivityAttributionMetric if kw.pop("sensitivity", False) else TaylorAttributionMetric
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    old = os.environ.get("TORCHPRUNER_GRAPHS")
    os.environ["TORCHPRUNER_GRAPHS"] = env
    try:
        return metric(model, DeviceLoader(x, y, B), F.cross_entropy, x.device, **kw).run_many(convs, True)
    finally:
        if old is None:
            del os.environ["TORCHPRUNER_GRAPHS"]
        else:
            os.environ["TORCHPRUNER_GRAPHS"] = old


@pytest.mark.gpu
@pytest.mark.parametrize("sensitivity", [False, True])
def test_graphed_taylor_bit_identical(cuda, sensitivity):
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    eng, _ = maybe_engine(model, [find_best_module_for_attributions(model, c) for c in convs], F.cross_entropy, cuda)
    x = torch.randn(150, 3, 32, 32, device=cuda)  # 4 batches of 40 -> last one ragged (30)
    y = torch.randint(0, 10, (150,), device=cuda)
    ref = _scores(model, x, y, 40, "0", sensitivity=sensitivity)
    for _ in range(2):  # first run: eager + capture; second: pure replay
        got = _scores(model, x, y, 40, "1", sensitivity=sensitivity)
        for a, r in zip(got, ref):
            np.testing.assert_array_equal(a, r)
    assert any(k[0] != "seen" for k in eng._graphs), "no graph was captured"


@pytest.mark.gpu
def test_graph_invalidated_by_new_weights(cuda):
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(1)
    model = prunable_vgg16().to(cuda).eval()
    x = torch.randn(64, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (64,), device=cuda)
    _scores(model, x, y, 32, "1")
    _scores(model, x, y, 32, "1")  # graph captured and replayed
    with torch.no_grad():  # in-place BN change: version bump -> re-pack -> new graph
        bn = model.features[1]
        bn.weight.mul_(1.5)
        bn.running_mean.add_(0.1)
    got = _scores(model, x, y, 32, "1")
    ref = _scores(model, x, y, 32, "0")
    for a, r in zip(got, ref):
        np.testing.assert_array_equal(a, r)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["taylor", "sensitivity", "apoz"])
def test_two_stream_pipeline_bit_identical(cuda, which):
    """Small batches run two in flight on two HIP streams (attributions/base.py _BatchPipeline):
    the accumulated scores must equal the one-stream loop bit for bit (per-stream arenas, folds
    chained in batch order), including a ragged last batch (its own, sequential first run)."""
    from torchpruner_amd import APoZAttributionMetric, SensitivityAttributionMetric, TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(1)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(330, 3, 32, 32, device=cuda)  # 8 batches of 40 + a ragged 10
    y = torch.randint(0, 10, (330,), device=cuda)
    metric = {"taylor": TaylorAttributionMetric, "sensitivity": SensitivityAttributionMetric,
              "apoz": APoZAttributionMetric}[which]
    out = {}
    for env in ("0", "1"):
        old = os.environ.get("TORCHPRUNER_STREAMS")
        os.environ["TORCHPRUNER_STREAMS"] = env
        try:
            out[env] = metric(model, DeviceLoader(x, y, 40), F.cross_entropy, cuda).run_many(convs, True)
        finally:
            if old is None:
                del os.environ["TORCHPRUNER_STREAMS"]
            else:
                os.environ["TORCHPRUNER_STREAMS"] = old
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("sensitivity", [False, True])
def test_pipelined_graph_replay_bit_identical(cuda, sensitivity):
    """Default (TORCHPRUNER_GRAPHS=auto): pipelined small batches replay one captured graph per
    stream slot (each into its own score arena); scores equal the eager one-stream loop bit for
    bit, including a ragged last batch, on the capturing run and on a pure-replay rerun."""
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(2)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    eng, _ = maybe_engine(model, [find_best_module_for_attributions(model, c) for c in convs], F.cross_entropy, cuda)
    x = torch.randn(430, 3, 32, 32, device=cuda)  # 10 batches of 40 + a ragged 30
    y = torch.randint(0, 10, (430,), device=cuda)
    old = os.environ.get("TORCHPRUNER_STREAMS")
    os.environ["TORCHPRUNER_STREAMS"] = "0"
    try:
        ref = _scores(model, x, y, 40, "0", sensitivity=sensitivity)
    finally:
        if old is None:
            del os.environ["TORCHPRUNER_STREAMS"]
        else:
            os.environ["TORCHPRUNER_STREAMS"] = old
    for _ in range(2):
        got = _scores(model, x, y, 40, "auto", sensitivity=sensitivity)
        for a, r in zip(got, ref):
            np.testing.assert_array_equal(a, r)
    graphs = [k for k in eng._graphs if k[0] != "seen"]
    assert len({k[-1] for k in graphs}) == 4, "one graph per pipeline slot (score arena), 4 slots by default"


@pytest.mark.gpu
def test_pipelined_apoz_graph_replay_matches_eager(cuda):
    """Fused-chain APoZ: pipelined batches replay one graph per slot (count buffers are graph
    outputs, re-zeroed inside the graph); the counts equal the one-stream eager loop exactly."""
    from torchpruner_amd import APoZAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.engine import maybe_engine
    from torchpruner_amd.models import prunable_vgg16
    from torchpruner_amd.utils import find_best_module_for_attributions
    torch.manual_seed(3)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    eng, _ = maybe_engine(model, [find_best_module_for_attributions(model, c) for c in convs], F.cross_entropy, cuda,
                          need_ce=False)
    x = torch.randn(450, 3, 32, 32, device=cuda)  # 11 batches of 40 + a ragged 10
    y = torch.randint(0, 10, (450,), device=cuda)
    out = {}
    for env in ("0", "1"):
        old = os.environ.get("TORCHPRUNER_STREAMS")
        os.environ["TORCHPRUNER_STREAMS"] = env
        try:
            for _ in range(2 if env == "1" else 1):
                out[env] = APoZAttributionMetric(model, DeviceLoader(x, y, 40), F.cross_entropy, cuda).run_many(
                    convs, True)
        finally:
            if old is None:
                del os.environ["TORCHPRUNER_STREAMS"]
            else:
                os.environ["TORCHPRUNER_STREAMS"] = old
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)
    assert any(k[0] == "apoz" for k in eng._graphs), "no APoZ graph was captured"


@pytest.mark.gpu
@pytest.mark.parametrize("layer", [0, 6, 9])
def test_shapley_graphed_prefix_chunks_bit_identical(cuda, layer):
    """Shapley on the fused engine replays one graph per prefix-chunk size (the prefix offset
    enters as a shifted rank vector): scores equal the eager launches bit for bit, on the
    capturing run and on a pure-replay rerun (ragged last chunk included)."""
    from torchpruner_amd import ShapleyAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(4)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    x = torch.randn(120, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (120,), device=cuda)

    def run(env):
        old = os.environ.get("TORCHPRUNER_GRAPHS")
        os.environ["TORCHPRUNER_GRAPHS"] = env
        try:
            np.random.seed(0)
            m = ShapleyAttributionMetric(model, DeviceLoader(x, y, 40), F.cross_entropy, cuda, sv_samples=2)
            return m.run(convs[layer], find_best_evaluation_module=True)
        finally:
            if old is None:
                del os.environ["TORCHPRUNER_GRAPHS"]
            else:
                os.environ["TORCHPRUNER_GRAPHS"] = old

    ref = run("0")
    for _ in range(2):
        np.testing.assert_array_equal(run("auto"), ref)


@pytest.mark.gpu
def test_invalidate_after_data_edit(cuda):
    """``param.data`` in-place edits bypass the version counter the engines key their packed
    weights on; ``engine.invalidate(model)`` drops the cached engine (and its graphs)."""
    from torchpruner_amd.engine import invalidate
    from torchpruner_amd.models import prunable_vgg16
    torch.manual_seed(5)
    model = prunable_vgg16().to(cuda).eval()
    x = torch.randn(64, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (64,), device=cuda)
    _scores(model, x, y, 16, "auto")
    model.features[0].weight.data.mul_(1.7)  # no version bump
    assert invalidate(model)
    got = _scores(model, x, y, 16, "auto")
    ref = _scores(model, x, y, 16, "0")
    for a, r in zip(got, ref):
        np.testing.assert_array_equal(a, r)


@pytest.mark.timeout(120)
def test_graph_capture_survives_a_pinning_loader_thread(cuda, monkeypatch):
    """A torch DataLoader with workers and pin_memory runs a pinning thread in this process while
    the engine captures its per-slot HIP graphs: with the default global capture mode that
    thread's host-memory calls invalidated the capture (hipErrorStreamCaptureInvalidated, found
    with one launch per batch, round 5); captures are thread-local now."""
    import torch.nn.functional as F

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.models import prunable_vgg16
    monkeypatch.setenv("TORCHPRUNER_COALESCE", "0")
    torch.manual_seed(0)
    model = prunable_vgg16().to(cuda).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    ds = torch.utils.data.TensorDataset(torch.randn(24 * 16, 3, 32, 32), torch.randint(0, 10, (24 * 16,)))
    dl = torch.utils.data.DataLoader(ds, batch_size=16, num_workers=1, pin_memory=True)
    got = TaylorAttributionMetric(model, dl, F.cross_entropy, cuda).run_many(convs, True)
    ref = TaylorAttributionMetric(model, [(x, y) for x, y in dl], F.cross_entropy, cuda).run_many(convs, True)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
