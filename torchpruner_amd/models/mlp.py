"""Fully-connected and small conv models of the reference experiments.

* :class:`FCNet` — MNIST / CIFAR-10 MLP ``Flatten -> Linear(in,2024) -> LeakyReLU ->
  Linear(2024,2024) -> LeakyReLU -> Linear(2024,10)`` with ``forward_partial``
  (experiments/models/mnist.py:9-35, cifar10.py:10-36). MNIST: 5,707,690 parameters
  (nbUNT:88); CIFAR-10: 10,338,602 (nbUNT:224).
* :class:`FMNISTConvNet` — conv5x5(32)/pool/conv3x3 p2(64)/pool/FC 4096/FC 10
  (experiments/models/fmnist.py:9-73), with the modern ``forward_partial`` protocol instead
  of the reference's older ``return_intermediate_output_module`` keywords (both accepted),
  and its hand-written pruning graph. Like the reference, ``bn1..bn3`` are registered but
  never executed.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from .partial import PartialForwardMixin, run_stages


class FCNet(nn.Module, PartialForwardMixin):
    def __init__(self, in_features=28 * 28, hidden=2024, num_classes=10):
        super().__init__()
        self.fc = nn.Sequential(
            nn.Flatten(1),
            nn.Linear(in_features, hidden),
            nn.LeakyReLU(),
            nn.Linear(hidden, hidden),
            nn.LeakyReLU(),
            nn.Linear(hidden, num_classes),
        )

    def _stages(self):
        return list(self.fc.children())

    def forward(self, x):
        return self.fc(x)

    def get_pruning_graph(self):
        layers = list(self.fc.children())
        return [(layers[3], [layers[5]]), (layers[1], [layers[3]])]


def mnist_fc():
    return FCNet(28 * 28)


def cifar10_fc():
    return FCNet(32 * 32 * 3)


class FMNISTConvNet(nn.Module, PartialForwardMixin):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, kernel_size=5, stride=1, padding=2)
        self.bn1 = nn.BatchNorm2d(32)
        self.relu1 = nn.ReLU()
        self.maxpool1 = nn.MaxPool2d(kernel_size=2)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=3, stride=1, padding=2)
        self.bn2 = nn.BatchNorm2d(64)
        self.relu2 = nn.ReLU()
        self.maxpool2 = nn.MaxPool2d(kernel_size=2)
        self.flatten = nn.Flatten(1)
        self.fc1 = nn.Linear(4096, 4096)
        self.bn3 = nn.BatchNorm1d(4096)
        self.relu3 = nn.ReLU()
        self.fc2 = nn.Linear(4096, 10)

    def _stages(self):
        return [self.conv1, self.relu1, self.maxpool1, self.conv2, self.relu2, self.maxpool2, self.flatten,
                self.fc1, self.relu3, self.fc2]

    def forward(self, x, return_intermediate_output_module=None, process_as_intermediate_output_module=None,
                linearize=False):
        if not linearize:
            return run_stages(self._stages(), x, to_module=return_intermediate_output_module,
                              from_module=process_as_intermediate_output_module)
        # "linearize": skip ReLUs and replace max-pool by avg-pool (fmnist.py:59-65)
        stages = []
        for m in self._stages():
            if m in (self.relu1, self.relu2, self.relu3):
                continue
            stages.append((lambda t: F.avg_pool2d(t, 2)) if m in (self.maxpool1, self.maxpool2) else m)
        return run_stages(stages, x)

    def get_pruning_graph(self):
        return [(self.fc1, [self.fc2]), (self.conv2, [self.fc1]), (self.conv1, [self.conv2])]
