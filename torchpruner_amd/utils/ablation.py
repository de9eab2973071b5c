"""Layerwise-robustness ablation (reference nbVGG:1233-1285 and the AUC of nbVGG:1521-1527).

The notebook removes units one at a time in ranking order (``z.index_fill_(1,[i],0)``) and
runs ``forward_partial`` after every removal: n sequential forwards plus two host syncs per
step. Removing the first p units of a ranking is exactly a Shapley prefix, so here K prefixes
are stacked by one ``ops.prefix_mask`` launch and evaluated by one forward (the fused HIP
engine when the model supports it, otherwise the model's own ``forward_partial``).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..engine import maybe_engine


@torch.no_grad()
def ablation_curve(model, eval_module, ranking, x, y, criterion=F.cross_entropy, max_eval_elements=1 << 29):
    """Loss and accuracy after removing the first p units of ``ranking``, p = 0..n.

    Returns ``(losses, accs)`` NumPy arrays of length n+1 (index 0 = nothing removed).
    """
    ranking = np.asarray(ranking)
    n = len(ranking)  # may be a partial ranking: units not listed are never removed
    B = x.shape[0]
    fused = maybe_engine(model, [eval_module], criterion, x.device)
    if fused is not None:
        engine, (k,) = fused
        zk, _ = engine.forward(x, stop_after=k)
        z = zk.permute(0, 3, 1, 2)  # channels_last view of the engine's NHWC activation

        def logits_of(masked):
            return engine.forward_from(k, masked.permute(0, 2, 3, 1))
    else:
        z = model.forward_partial(x, to_module=eval_module).contiguous()

        def logits_of(masked):
            return model.forward_partial(masked, from_module=eval_module)
    units = z.shape[1]
    rank_of = torch.full((units,), units + 1, dtype=torch.int32)
    rank_of[torch.as_tensor(ranking, dtype=torch.long)] = torch.arange(n, dtype=torch.int32)
    rank_of = rank_of.to(x.device)
    per = max(1, z[0].numel())
    K = max(1, int(max_eval_elements // (4 * B * per)))
    losses, accs = [], []
    p = 0
    while p <= n:
        cnt = min(K, n + 1 - p)
        masked = ops.prefix_mask(z, rank_of, p, cnt)
        logits = logits_of(masked).reshape(cnt * B, -1)
        yy = y.repeat(cnt)
        # criterion contract (README): accepts reduction="none" -> per-sample; mean per prefix
        loss = criterion(logits, yy, reduction="none").reshape(cnt, B).mean(1)
        acc = (logits.argmax(-1) == yy).float().reshape(cnt, B).mean(1)
        losses.append(loss)
        accs.append(acc)
        p += cnt
    return torch.cat(losses).cpu().numpy(), torch.cat(accs).cpu().numpy()


def ablation_auc(losses) -> float:
    """Mean increase of the loss over the removal curve (nbVGG:1521-1527): lower is better."""
    losses = np.asarray(losses, dtype=np.float64)
    n = len(losses) - 1
    return float(np.sum(losses[1:] - losses[0]) / max(n, 1))
