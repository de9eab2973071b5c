"""Reference module path alias (TorchPruner's pruner/opt_pruner.py) -> the MI355X implementation."""
from torchpruner_amd.pruner.opt_pruner import OptimizerPruner  # noqa: F401
