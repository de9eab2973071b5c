from .graph import (
    ACTIVATIONS,
    discover_cascade,
    find_best_module_for_attributions,
    get_resnet_pruning_graph,
    get_vgg_pruning_graph,
)
from .flops import count_parameters, count_flops
from .train import recalibrate_bn, test, train

__all__ = [
    "ACTIVATIONS",
    "discover_cascade",
    "find_best_module_for_attributions",
    "get_resnet_pruning_graph",
    "get_vgg_pruning_graph",
    "count_parameters",
    "count_flops",
    "train",
    "test",
    "recalibrate_bn",
]
