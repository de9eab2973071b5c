"""Reference module path alias (TorchPruner's attributions/methods/apoz.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.apoz import APoZAttributionMetric  # noqa: F401
