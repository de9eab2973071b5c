"""VGG-BN for CIFAR-10 (reference: experiments/models/cifar10.py:39-77).

The reference builds torchvision's ``vgg16_bn(num_classes)``, replaces the classifier by
``Dropout, Linear(512,512), ReLU(True), Dropout, Linear(512,512), ReLU(True), Linear(512,10)``
and monkey-patches ``VGG.forward = VGG.forward_partial`` so the model skips ``avgpool``
(for 32x32 inputs the features end at 512x1x1). torchvision is not available here, so the
network is defined directly with the same module tree: the ``state_dict`` keys
(``features.0.weight``, ``features.1.running_mean``, ..., ``classifier.6.bias``) and the
parameter count (15,253,578 for VGG16-BN, nbVGG:167) match the reference model.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .partial import PartialForwardMixin

CFGS = {
    "vgg11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}


def make_features(cfg, batch_norm=True, in_channels=3) -> nn.Sequential:
    layers = []
    c = in_channels
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers.append(nn.Conv2d(c, v, kernel_size=3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2d(v))
            layers.append(nn.ReLU(inplace=True))
            c = v
    return nn.Sequential(*layers)


class VGG(nn.Module, PartialForwardMixin):
    """torchvision-layout VGG whose forward == forward_partial (skips avgpool, like the reference)."""

    def __init__(self, features: nn.Sequential, num_classes=10, hidden=512, init_weights=True):
        super().__init__()
        self.features = features
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))  # registered for layout parity; unused (reference quirk)
        self.classifier = nn.Sequential(
            nn.Dropout(),
            nn.Linear(512, hidden),
            nn.ReLU(True),
            nn.Dropout(),
            nn.Linear(hidden, hidden),
            nn.ReLU(True),
            nn.Linear(hidden, num_classes),
        )
        if init_weights:
            self._initialize_weights()

    def _stages(self):
        return list(self.features.children()) + [_flatten] + list(self.classifier.children())

    def forward(self, x, to_module=None, from_module=None):
        return self.forward_partial(x, to_module=to_module, from_module=from_module)

    def _initialize_weights(self):
        # torchvision VGG._initialize_weights
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.constant_(m.bias, 0)


def _flatten(x):
    return torch.flatten(x, 1)


def vgg_cifar(depth: int = 16, num_classes: int = 10, batch_norm: bool = True) -> VGG:
    return VGG(make_features(CFGS[f"vgg{depth}"], batch_norm=batch_norm), num_classes=num_classes)


def prunable_vgg16(num_classes: int = 10) -> VGG:
    """VGG16-BN for CIFAR with the reference's classifier (cifar10.py:62-77)."""
    return vgg_cifar(16, num_classes)


def get_vgg_model_with_name():
    return prunable_vgg16(), "CIFAR10-VGG16"
