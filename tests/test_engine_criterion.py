"""Criterion plumbing of the native engines (CPU): dL/dlogits through autograd for a user
criterion and per-sample losses with the reference's reduction="none" convention."""
import torch
import torch.nn.functional as F

from torchpruner_amd.engine.fused_chain import engine_criterion, logits_grad, per_sample_loss


def _mse_onehot(out, y, reduction="mean"):
    return F.mse_loss(out, F.one_hot(y, out.shape[1]).float(), reduction=reduction)


def test_engine_criterion_detects_cross_entropy():
    assert engine_criterion(F.cross_entropy, "cpu") is None
    assert engine_criterion(torch.nn.CrossEntropyLoss(), "cpu") is None
    assert engine_criterion(_mse_onehot, "cpu") is _mse_onehot
    ls = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
    assert engine_criterion(ls, "cpu") is ls  # not plain CE: differentiated by autograd


def test_logits_grad_matches_autograd_of_the_batch_loss():
    torch.manual_seed(0)
    logits = torch.randn(6, 5)
    y = torch.randint(0, 5, (6,))
    for crit in (_mse_onehot, torch.nn.CrossEntropyLoss(label_smoothing=0.2)):
        lg = logits.clone().requires_grad_(True)
        crit(lg, y).backward()
        torch.testing.assert_close(logits_grad(logits, y, crit), lg.grad)


def test_per_sample_loss_sums_trailing_dims():
    torch.manual_seed(1)
    logits = torch.randn(4, 3)
    y = torch.randint(0, 3, (4,))
    got = per_sample_loss(logits, y, _mse_onehot)
    ref = ((logits - F.one_hot(y, 3).float()) ** 2).sum(1)
    torch.testing.assert_close(got, ref)
    yt = torch.randn(4, 1)
    got2 = per_sample_loss(logits[:, :1], yt, F.mse_loss)
    torch.testing.assert_close(got2, ((logits[:, :1] - yt) ** 2).reshape(4))
