"""Reference module path alias (TorchPruner's attributions/methods/sensitivity.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.sensitivity import SensitivityAttributionMetric  # noqa: F401
