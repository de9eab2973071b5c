"""Reference module path alias (TorchPruner's utils/graph.py) -> the MI355X implementation."""
from torchpruner_amd.utils.graph import ACTIVATIONS, find_best_module_for_attributions, get_vgg_pruning_graph  # noqa: F401
