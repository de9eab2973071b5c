"""Reference module path alias (TorchPruner's attributions/methods/random.py) -> the MI355X implementation."""
from torchpruner_amd.attributions.methods.random import RandomAttributionMetric  # noqa: F401
