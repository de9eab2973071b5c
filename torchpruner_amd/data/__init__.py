"""Data: synthetic on-device datasets shaped like the reference's CIFAR-10 / MNIST / ImageNet, and
the real CIFAR-10 / MNIST / Fashion-MNIST binary files resident in HBM with GPU augmentation."""
from .datasets import (DeviceDataLoader, DeviceImageDataset, augment_batch, get_dataset_and_loaders, read_cifar10,
                       read_mnist)
from .prefetch import prefetch_to_device
from .synthetic import (SHAPES, DeviceLoader, PrototypeTask, ShardLoader, StreamLoader, TaskStream, loaders,
                        synthetic_dataset, teacher_labels)

__all__ = ["SHAPES", "DeviceLoader", "PrototypeTask", "ShardLoader", "StreamLoader", "TaskStream", "loaders",
           "prefetch_to_device", "synthetic_dataset", "teacher_labels", "DeviceDataLoader", "DeviceImageDataset",
           "augment_batch", "get_dataset_and_loaders", "read_cifar10", "read_mnist"]
