"""Reference module path alias (TorchPruner's attributions/methods/taylor.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.taylor import TaylorAttributionMetric  # noqa: F401
