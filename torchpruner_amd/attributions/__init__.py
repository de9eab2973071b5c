"""Attribution metrics (API parity with reference torchpruner/attributions/__init__.py:1-7)."""
from .base import _AttributionMetric, ScoreAccumulator, SUPPORTED_OUT_PRUNING_MODULES
from .methods.random import RandomAttributionMetric
from .methods.weight_norm import WeightNormAttributionMetric
from .methods.apoz import APoZAttributionMetric
from .methods.sensitivity import SensitivityAttributionMetric
from .methods.taylor import TaylorAttributionMetric
from .methods.shapley import ShapleyAttributionMetric
from ..utils.graph import find_best_module_for_attributions

__all__ = [
    "RandomAttributionMetric",
    "WeightNormAttributionMetric",
    "APoZAttributionMetric",
    "SensitivityAttributionMetric",
    "TaylorAttributionMetric",
    "ShapleyAttributionMetric",
    "find_best_module_for_attributions",
]
