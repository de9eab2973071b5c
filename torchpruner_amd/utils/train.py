"""Training / evaluation loops (reference: experiments/utils/train.py:11-72), data-parallel aware.

``train`` and ``test`` keep the reference's signatures and return values. In a live process
group ``test`` all-reduces its correct/total/loss counters (R8) so every rank reports the
global accuracy; ``train`` expects the model to be wrapped in DistributedDataParallel by the
caller (see :mod:`torchpruner_amd.parallel.ddp`) and the loader to be sharded.
"""
from __future__ import annotations

import logging
from timeit import default_timer as timer

import torch

from ..data.prefetch import prefetch_to_device
from ..parallel import dist as pdist

logger = logging.getLogger("torchpruner")


def _batches(loader, rank, world, shard):
    if shard and world > 1:
        yield from ((x, y) for _, x, y in pdist.ShardedBatches(loader, rank, world))
    else:
        yield from loader


def train(model, device, loss, train_loader, optimizer, epoch, log_every=20, shard=True, max_steps=None):
    """One epoch of SGD; returns (average loss, accuracy) over this rank's samples."""
    model.train()
    correct = samples = 0
    cumulative_loss = 0.0
    start = timer()
    world, rank = pdist.get_world_size(), pdist.get_rank()
    for batch_idx, (data, target) in enumerate(prefetch_to_device(_batches(train_loader, rank, world, shard), device)):
        if max_steps is not None and batch_idx >= max_steps:
            break
        optimizer.zero_grad(set_to_none=True)
        output = model(data)
        curr_loss = loss(output, target)
        curr_loss.backward()
        optimizer.step()
        with torch.no_grad():
            cumulative_loss += curr_loss.detach() * len(target)
            correct += (output.argmax(1) == target.view(-1)).sum()
        samples += len(target)
        if log_every and batch_idx % log_every == 0:
            logger.info("Train Epoch: %d [%d] loss %.6f acc %.3f time %.1fs", epoch, batch_idx * len(data),
                        float(curr_loss), float(correct) / max(samples, 1), timer() - start)
            start = timer()
    return float(cumulative_loss) / max(samples, 1), float(correct) / max(samples, 1)


@torch.no_grad()
def recalibrate_bn(model, batches, max_batches=None) -> int:
    """Re-estimate the BatchNorm running statistics of a (freshly pruned) model.

    Pruning a layer's filters removes input channels of the next conv, so the running mean /
    variance of the BN after it no longer describe its input and eval-mode accuracy collapses
    until training re-adapts them (momentum 0.1: ~20 steps). This resets every BN's running
    statistics and re-accumulates them as an exact cumulative average over ``batches`` (inputs,
    or (x, y) pairs) in training mode, without gradients; other modules (Dropout) stay in eval
    mode. Feed every data-parallel rank the same batches to keep replicas identical. Returns
    the number of batches used."""
    from torch.nn.modules.batchnorm import _BatchNorm
    bns = [m for m in model.modules() if isinstance(m, _BatchNorm) and m.track_running_stats]
    if not bns:
        return 0
    was = model.training
    saved = [(m, m.momentum, m.training) for m in bns]
    model.eval()
    for m in bns:
        m.reset_running_stats()
        m.momentum = None  # cumulative moving average
        m.train()
    n = 0
    try:
        for b in batches:
            if max_batches is not None and n >= max_batches:
                break
            x = b[0] if isinstance(b, (tuple, list)) else b
            model(x)
            n += 1
    finally:
        for m, mom, tr in saved:
            m.momentum = mom
            m.train(tr)
        model.train(was)
    return n


@torch.no_grad()
def test(model, device, loss, test_loader, verbose=1, shard=False, native=True):
    """Eval-mode average loss and accuracy (reference train.py:51-72). ``native``: logits come
    from the HIP engines when the model lowers to one (same fp32 semantics, no library GEMMs)."""
    from ..engine import native_logits
    model.eval()
    cum = torch.zeros(3, dtype=torch.float64, device=device)  # loss*n, correct, n
    world, rank = pdist.get_world_size(), pdist.get_rank()
    for data, target in prefetch_to_device(_batches(test_loader, rank, world, shard), device):
        output = native_logits(model, data) if native else None
        if output is None:
            output = model(data)
        cum[0] += loss(output, target).double() * len(target)
        cum[1] += (output.argmax(1) == target.view(-1)).sum()
        cum[2] += len(target)
    if shard and world > 1:
        pdist.all_reduce_sum_(cum)
    avg_loss, acc = float(cum[0] / cum[2].clamp_min(1)), float(cum[1] / cum[2].clamp_min(1))
    if verbose > 0:
        logger.info("Test set: Average loss: %.4f, Accuracy: %d/%d (%.3f%%)", avg_loss, int(cum[1]), int(cum[2]),
                    100.0 * acc)
    return avg_loss, acc
