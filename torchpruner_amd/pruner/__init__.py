"""Structured pruner (API parity with reference torchpruner/pruner/__init__.py:1)."""
from .pruner import Pruner, SUPPORTED_IN_PRUNING_MODULES, SUPPORTED_OUT_PRUNING_MODULES
from .opt_pruner import OptimizerPruner

__all__ = ["Pruner", "OptimizerPruner", "SUPPORTED_IN_PRUNING_MODULES", "SUPPORTED_OUT_PRUNING_MODULES"]
