"""torchpruner_amd — MI355X-native structured-pruning engine.

Same public API as TorchPruner (``torchpruner.attributions``, ``torchpruner.pruner``,
``torchpruner.utils``) with gfx950 HIP kernels for the hot paths and RCCL data parallelism.
The top-level re-exports match what the reference's notebooks import
(``from torchpruner import Pruner, ShapleyAttributionMetric, ...``).
"""
__version__ = "0.1.0"

from .attributions import (
    APoZAttributionMetric,
    RandomAttributionMetric,
    SensitivityAttributionMetric,
    ShapleyAttributionMetric,
    TaylorAttributionMetric,
    WeightNormAttributionMetric,
)
from .pruner import OptimizerPruner, Pruner
from .utils import find_best_module_for_attributions, get_resnet_pruning_graph, get_vgg_pruning_graph

__all__ = [
    "APoZAttributionMetric",
    "RandomAttributionMetric",
    "SensitivityAttributionMetric",
    "ShapleyAttributionMetric",
    "TaylorAttributionMetric",
    "WeightNormAttributionMetric",
    "OptimizerPruner",
    "Pruner",
    "find_best_module_for_attributions",
    "get_resnet_pruning_graph",
    "get_vgg_pruning_graph",
]
