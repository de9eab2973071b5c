"""Reference module path alias (TorchPruner's attributions/attributions.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.base import ACTIVATIONS, SUPPORTED_OUT_PRUNING_MODULES, _AttributionMetric  # noqa: F401
