"""The fp64 oracle of the fused engine's scores (engine/oracle.py) on the CPU: its plain mode equals
autograd Taylor / Sensitivity of the reference semantics, and its mask-conditioned mode equals the
plain one when the emulated engine takes fp64's own decisions."""
import numpy as np
import torch
import torch.nn.functional as F

from torchpruner_amd import SensitivityAttributionMetric, TaylorAttributionMetric
from torchpruner_amd.data import DeviceLoader
from torchpruner_amd.engine.fused_chain import build_plan
from torchpruner_amd.engine.oracle import engine_scores_fp64
from torchpruner_amd.models import vgg_cifar
from torchpruner_amd.utils import find_best_module_for_attributions


class _TorchChain:
    """Minimal stand-in for FusedChainEngine.forward in fp64 torch (engine layouts: NHWC acts,
    uint8 pool argmax q = 2*dy + dx, (B,1,1,F) linear activations)."""

    def __init__(self, model):
        self.plan, why = build_plan(model)
        assert self.plan is not None, why

    def forward(self, x):
        h = x.double()
        acts = []
        for blk in self.plan.convs:
            h = F.batch_norm(F.conv2d(h, blk.conv.weight, blk.conv.bias, padding=1), blk.bn.running_mean,
                             blk.bn.running_var, blk.bn.weight, blk.bn.bias, False, 0.0, blk.bn.eps)
            am = None
            if blk.pool is not None:
                B, C, H, W = h.shape
                win = h.view(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
                h, q = win.max(-1)
                am = q.to(torch.uint8).permute(0, 2, 3, 1).contiguous()
            h = torch.relu(h)
            acts.append((h.permute(0, 2, 3, 1).contiguous(), am))
        lin = [h.reshape(h.shape[0], 1, 1, -1)]
        for lb in self.plan.linears:
            z = F.linear(lin[-1], lb.linear.weight, lb.linear.bias)
            lin.append(torch.relu(z) if lb.relu is not None else z)
        return lin[-1].reshape(x.shape[0], -1), {"acts": acts, "lin_acts": lin}


def _model():
    torch.manual_seed(1)
    m = vgg_cifar(11).double().eval()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.1, 0.1)
            if isinstance(mod, torch.nn.Linear):
                mod.weight.normal_(0, 0.05)
    return m


def test_oracle_matches_autograd_reference():
    m = _model()
    eng = _TorchChain(m)
    x = torch.randn(6, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (6,))
    mods = [mm for mm in m.features if isinstance(mm, torch.nn.Conv2d)] + [m.classifier[1], m.classifier[4]]
    for mode, cls in (("taylor", TaylorAttributionMetric), ("sensitivity", SensitivityAttributionMetric)):
        ref = cls(m, DeviceLoader(x, y, 6), F.cross_entropy, "cpu", reduction="none").run_many(mods, True)
        if mode == "taylor":  # the reference takes |.| per sample unless signed
            ref_s = cls(m, DeviceLoader(x, y, 6), F.cross_entropy, "cpu", reduction="none",
                        signed=True).run_many(mods, True)
        plain, flips = engine_scores_fp64(eng, x, y, conditioned=False, mode=mode)
        cond, _ = engine_scores_fp64(eng, x, y, conditioned=True, mode=mode)
        assert all(v == 0 for v in flips.values()), flips
        for k, mm in enumerate(mods):
            b = eng.plan.blocks.index(next(bb for bb in eng.plan.blocks
                                           if bb.relu is find_best_module_for_attributions(m, mm)))
            got = plain[b].numpy()
            # the reference path returns float32 scores (API contract): compare at fp32 precision
            tol = 1e-6 * np.abs(ref[k]).max()
            np.testing.assert_allclose(np.abs(got) if mode == "taylor" else got, ref[k], rtol=1e-5, atol=tol)
            if mode == "taylor":
                np.testing.assert_allclose(got, ref_s[k], rtol=1e-5, atol=tol)
            assert torch.equal(cond[b], plain[b])


def test_oracle_counts_and_replays_flipped_decisions():
    """A decision the engine takes differently (here: one ReLU unit forced off) is counted and the
    conditioned oracle follows the engine, not fp64."""
    m = _model()
    eng = _TorchChain(m)
    x = torch.randn(4, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (4,))
    fwd = eng.forward

    def flipped(xx):
        logits, saved = fwd(xx)
        h, am = saved["acts"][2]
        h = h.clone()
        pos = (h > 0).nonzero()[0]
        h[tuple(pos)] = 0.0
        saved["acts"][2] = (h, am)
        return logits, saved

    eng.forward = flipped
    plain, flips = engine_scores_fp64(eng, x, y, conditioned=False)
    cond, flips2 = engine_scores_fp64(eng, x, y, conditioned=True)
    # plain fp64 follows its own decisions, so downstream of the flip it agrees with the engine
    assert flips[2] == 1 and sum(flips.values()) == 1 and flips2[2] == 1
    assert not torch.equal(cond[0], plain[0])  # upstream scores follow the engine's mask


def test_flip_bound_catches_a_wrong_relu_threshold():
    """Red on purpose: an engine whose ReLU decides ``x > 0.02`` instead of ``x > 0`` (a
    systematic mis-decision near zero) still matches the mask-conditioned oracle exactly — the
    tight check conditions on the engine's own decisions — but its flips break the per-block
    bound (oracle.flip_bound: the rounding-tie rate plus a Poisson allowance) that the GPU test and
    smoke() assert."""
    from torchpruner_amd.engine.oracle import flip_bound, flip_violations
    m = _model()
    x = torch.randn(4, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (4,))
    good = _TorchChain(m)
    tot = {}
    _, flips = engine_scores_fp64(good, x, y, conditioned=True, totals=tot)
    assert set(tot) == set(flips) and all(v > 0 for v in tot.values())
    assert flip_violations(flips, tot) == {}
    bad = _TorchChain(m)
    fwd = bad.forward

    def thresholded(xx):
        logits, saved = fwd(xx)
        saved["acts"] = [(torch.where(h > 0.02, h, torch.zeros((), dtype=h.dtype)), am) for h, am in saved["acts"]]
        return logits, saved

    bad.forward = thresholded
    tot2 = {}
    _, flips2 = engine_scores_fp64(bad, x, y, conditioned=True, totals=tot2)
    viol = flip_violations(flips2, tot2)
    assert viol, flips2
    assert all(f > flip_bound(n) for f, n in viol.values())
    print({b: (f, n, round(flip_bound(n), 1)) for b, (f, n) in viol.items()})
