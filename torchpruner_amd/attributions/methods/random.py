"""Random baseline (reference: methods/random.py:5-13)."""
import numpy as np

from ..base import _AttributionMetric


class RandomAttributionMetric(_AttributionMetric):
    """Uniform random scores; ignores ``reduction``. Uses NumPy's global RNG like the reference."""

    def run(self, module, **kwargs):
        module = super().run(module, **kwargs)
        n = module.weight.shape[0]  # output dimension
        return np.random.random((n,))

    def find_evaluation_module(self, module, find_best_evaluation_module=False):
        # needs a module with weights
        return module
