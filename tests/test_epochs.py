"""Engine cache epochs (engine/epochs.py): every torch.optim step moves the key, whatever the
optimizer implementation (fused kernels leave autograd version counters alone)."""
import torch

from torchpruner_amd.engine import epochs


def test_optimizer_step_moves_engine_key():
    p = torch.nn.Parameter(torch.randn(8))
    for opt in (torch.optim.SGD([p], lr=0.1, momentum=0.9), torch.optim.Adam([p], lr=0.1)):
        p.grad = torch.ones(8)
        k0 = epochs.engine_key()
        opt.step()
        assert epochs.engine_key() != k0


def test_stats_and_forward_epochs():
    k0 = epochs.engine_key()
    epochs.bump_stats()
    assert epochs.engine_key() != k0
    f0 = epochs.FWD[0]
    m = torch.nn.Linear(2, 2)
    m.register_forward_pre_hook(epochs.bump_fwd)
    m(torch.randn(1, 2))
    assert epochs.FWD[0] == f0 + 1
