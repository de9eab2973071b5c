"""Reference module path alias (TorchPruner's attributions/methods/shapley_values.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.shapley import ShapleyAttributionMetric  # noqa: F401
