"""Experiment bookkeeping (reference: experiments/utils/utils.py:1-113).

``get_module_name``, ``get_layer_sizes``, ``get_parameter_count_and_flops`` (own FLOP counter
instead of thop), the CSV :class:`Logger` (with the reference's ``flops_full`` bug fixed:
utils.py:64 logs the parameter count there) and the plotting vocabulary (``COLORS``,
``METHODS_MAPPING``, ``map_method_vis``, ``format_plt`` when matplotlib is importable).
Only rank 0 writes in a process group.
"""
from __future__ import annotations

import csv
import os
from datetime import datetime

from ..parallel import dist as pdist
from .flops import count_flops


def now():
    return datetime.now().strftime("%Y%m%dT%H%M%S")


def get_module_name(model, module):
    for module_name, m in model.named_modules():
        if m is module:
            return module_name
    return None


def get_layer_sizes(model, graph=None):
    """'64-128-...' widths of the prunable layers (model.get_pruning_graph() or ``graph``)."""
    graph = graph if graph is not None else model.get_pruning_graph()
    return "-".join(str(m.weight.shape[0]) for m, _ in graph)


def get_parameter_count_and_flops(model, input_size, device):
    """(flops per sample, params); flops = 2 * MACs like the reference's 2*thop MACs."""
    return count_flops(model, input_size, device)


class Logger:
    """Append one CSV row per pruning step to ``{directory}/{name}.csv``."""

    FIELDS = ["timestamp", "epoch", "train_acc", "test_acc", "test_acc_pp", "train_loss", "test_loss",
              "test_loss_pp", "n_params", "flops", "n_params_full", "flops_full", "layers", "train_time",
              "prune_time", "experiment", "pr"]

    def __init__(self, name, model, model_input_size, device, directory="results", pr=None, graph=None):
        self.now = now()
        self.name = name
        self.pr = pr
        self.graph = graph
        self.input_size = model_input_size
        self.device = device
        self.flops_original, self.n_params_original = get_parameter_count_and_flops(model, model_input_size, device)
        self.filename = os.path.join(directory, f"{name}.csv")

    def log(self, model, test_loss, test_acc, test_loss_pp, test_acc_pp, prune_time, epoch=0, train_acc=0,
            train_loss=0, train_time=0.0):
        flops, n_params = get_parameter_count_and_flops(model, self.input_size, self.device)
        try:
            layers = get_layer_sizes(model, self.graph)
        except AttributeError:
            layers = ""
        row = {"timestamp": self.now, "epoch": epoch, "train_acc": train_acc, "test_acc": test_acc,
               "test_acc_pp": test_acc_pp, "train_loss": train_loss, "test_loss": test_loss,
               "test_loss_pp": test_loss_pp, "n_params": n_params, "flops": flops,
               "n_params_full": self.n_params_original, "flops_full": self.flops_original, "layers": layers,
               "train_time": train_time, "prune_time": prune_time, "experiment": self.name, "pr": self.pr}
        if pdist.get_rank() != 0:
            return row
        os.makedirs(os.path.dirname(self.filename) or ".", exist_ok=True)
        with open(self.filename, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self.FIELDS)
            if f.tell() == 0:
                w.writeheader()
            w.writerow(row)
        return row


COLORS = ["orange", "#4e79a7", "#59a14f", "#9c755f", "#666666", "#e15759", "#b07aa1", "#BEAD53", "grey"]

METHODS_MAPPING = {
    "SV mean+2std": ("SV, $\\mu+2\\sigma$ aggr.", COLORS[5]),
    "Random": ("Random", COLORS[0]),
    "Sensitivity": ("Saliency", COLORS[2]),
    "Taylor": ("Taylor", COLORS[1]),
    "APoZ": ("APoZ", COLORS[8]),
    "Weight Norm": ("$||w||_1$", COLORS[6]),
    "Taylor signed": ("Taylor (no abs)", COLORS[3]),
    "SV": ("SV, $\\mu$ aggr.", "black"),
}


def map_method_vis(method_name):
    return METHODS_MAPPING[method_name]


def format_plt(ax, title, xlabel, ylabel):
    import matplotlib.pyplot as plt  # optional dependency
    plt.sca(ax)
    plt.box(False)
    plt.tick_params(color="#222222", labelcolor="#222222")
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    plt.gca().yaxis.grid(True, linestyle="-", which="major", color="lightgrey", alpha=0.5)
    if title is not None:
        plt.title(title)
