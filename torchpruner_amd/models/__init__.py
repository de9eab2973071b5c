"""Model zoo with the ``forward_partial`` protocol (reference experiments/models/)."""
from .partial import PartialForwardMixin, SequentialPartial, run_stages, with_forward_partial
from .vgg import VGG, get_vgg_model_with_name, make_features, prunable_vgg16, vgg_cifar
from .resnet import ResNet, BasicBlock, Bottleneck, resnet18, resnet34, resnet50, resnet101, resnet152
from .mlp import FCNet, FMNISTConvNet, cifar10_fc, mnist_fc

__all__ = [
    "PartialForwardMixin", "SequentialPartial", "run_stages", "with_forward_partial",
    "VGG", "get_vgg_model_with_name", "make_features", "prunable_vgg16", "vgg_cifar",
    "ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
    "FCNet", "FMNISTConvNet", "cifar10_fc", "mnist_fc",
]
