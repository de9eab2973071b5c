"""Synthetic on-device datasets shaped like the reference's CIFAR-10 / MNIST / ImageNet."""
from .prefetch import prefetch_to_device
from .synthetic import SHAPES, DeviceLoader, PrototypeTask, ShardLoader, StreamLoader, TaskStream, loaders, synthetic_dataset, teacher_labels

__all__ = ["SHAPES", "DeviceLoader", "PrototypeTask", "ShardLoader", "StreamLoader", "TaskStream", "loaders", "prefetch_to_device",
           "synthetic_dataset", "teacher_labels"]
