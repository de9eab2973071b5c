import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torchpruner_amd import ops
    ops.require()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda")
