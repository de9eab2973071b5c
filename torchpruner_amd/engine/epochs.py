"""Counters that invalidate the engines' packed-weight caches where autograd version counters do
not move.

The attribution engines (fused_chain.FusedChainEngine, resnet_engine.ResNetEngine) and the
training convs' batched weight packs (train._PackSet) cache operands keyed by the parameters'
``_version``. Two in-place writers do not bump it (measured: scripts/probes/pack_cache_probe.py):

* torch's fused optimizers (``SGD(fused=True)``, ``Adam(fused=True)``) update parameters with one
  fused kernel that leaves the version counters alone -> ``OPT`` counts every torch.optim step
  (a global post-step hook, whatever the implementation);
* the native training BatchNorm kernels update ``running_mean`` / ``running_var`` through raw
  pointers -> ``STATS`` counts native training-BN forwards.

``FWD`` counts forwards of models given to ``enable_native_convs`` (covers optimizers outside
torch.optim for the training packs)."""
import torch.optim.optimizer as _optim

OPT = [0]
STATS = [0]
FWD = [0]


def _bump_opt(*_args, **_kw):
    OPT[0] += 1


def bump_fwd(*_args, **_kw):
    FWD[0] += 1


def bump_stats():
    STATS[0] += 1


def engine_key() -> tuple:
    """Epoch part of an engine's packed-weight cache key."""
    return (OPT[0], STATS[0])


_optim.register_optimizer_step_post_hook(_bump_opt)
