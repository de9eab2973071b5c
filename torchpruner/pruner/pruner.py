"""Reference module path alias (TorchPruner's pruner/pruner.py) -> the MI355X implementation."""
from torchpruner_amd.pruner.pruner import SUPPORTED_IN_PRUNING_MODULES, SUPPORTED_OUT_PRUNING_MODULES, Pruner  # noqa: F401
