"""Fused native execution engines (HIP kernels, no autograd) used by the attribution metrics
when the model/criterion/device allow it; everything else runs the generic hook path."""
from .fused_chain import FusedChainEngine, Plan, build_plan, criterion_is_cross_entropy, maybe_engine
from .resnet_engine import ResNetEngine, build_resnet_plan, maybe_resnet_engine

__all__ = ["FusedChainEngine", "Plan", "build_plan", "criterion_is_cross_entropy", "maybe_engine", "ResNetEngine",
           "build_resnet_plan", "maybe_resnet_engine"]
