"""L1 weight norm per output unit — Li et al., ICLR'17 (reference: methods/weight_norm.py:5-23).

The reference copies the full weight to the host and sums it with NumPy; here the row-L1 runs
on the device holding the weight (the HIP channel-reduction kernel, K9d: the weight viewed as
one "sample" with Cout channels) and only the (C,) result is copied.
"""
import torch

from ... import ops
from ..base import _AttributionMetric


class WeightNormAttributionMetric(_AttributionMetric):
    def run(self, module, **kwargs):
        module = super().run(module, **kwargs)
        with torch.no_grad():
            w = module.weight.detach()
            attr = ops.channel_reduce(None, w.reshape(1, w.shape[0], -1).float(), "sensitivity")[0]
        return attr.cpu().numpy()

    def find_evaluation_module(self, module, find_best_evaluation_module=False):
        # not meaningful after BN / activation: always the weight-carrying module
        return module
