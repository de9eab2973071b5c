"""Reference module path alias (TorchPruner's attributions/methods/weight_norm.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.weight_norm import WeightNormAttributionMetric  # noqa: F401
