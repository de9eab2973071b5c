"""fp64 oracles of the fused VGG engine's Taylor / Sensitivity scores.

A deep ReLU network is discontinuous in its inputs: a pre-activation within rounding of 0, or two
max-pool candidates within rounding of each other, makes the fp32 forward take a different ReLU
mask / pool argmax than the fp64 one, and every score upstream of that unit then differs by far
more than fp32 rounding. Comparing an fp32 kernel against a plain fp64 run therefore measures the
kernel's rounding *and* the conditioning of the input. This module separates the two:

``engine_scores_fp64(engine, x, y, conditioned=True)`` replays the fused engine's own discrete
decisions (every ReLU mask, every 2x2 max-pool argmax, read back from the engine's forward) in
an fp64 forward + input-gradient backward. The fused scores must match it to fp32 rounding of
the arithmetic alone, whatever the input. ``conditioned=False`` is the plain fp64 run (its own
masks and argmaxes), which the reference's semantics define (taylor.py:31-49,
attributions.py:58-68); ``decision_flips`` counts where the two runs' decisions differ.

Runs on the CPU in fp64 on one batch (the per-batch mean loss of the reference,
attributions.py:66): the caller loops batches and reduces.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(t, c):
    """Engine NHWC (padded width) -> NCHW fp64 CPU with the real ``c`` channels."""
    return t.permute(0, 3, 1, 2)[:, :c].double().cpu().contiguous()  # NCHW-contiguous: same conv algorithms


def _affine(blk):
    """Eval-mode BN folded into a per-channel (scale, shift) with the conv bias, in fp64."""
    conv, bn = blk.conv, blk.bn
    c = conv.out_channels
    bias = conv.bias.detach().double().cpu() if conv.bias is not None else torch.zeros(c, dtype=torch.float64)
    if bn is None:
        return torch.ones(c, dtype=torch.float64), bias
    inv = torch.rsqrt(bn.running_var.detach().double().cpu() + bn.eps)
    g = bn.weight.detach().double().cpu() if bn.weight is not None else torch.ones(c, dtype=torch.float64)
    b = bn.bias.detach().double().cpu() if bn.bias is not None else torch.zeros(c, dtype=torch.float64)
    scale = g * inv
    return scale, (bias - bn.running_mean.detach().double().cpu()) * scale + b


def _windows(pre):
    """(B, C, H, W) -> (B, C, H/2, W/2, 4) with q = 2*dy + dx (the engine's argmax byte)."""
    B, C, H, W = pre.shape
    return pre.view(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)


def _unpool(gp, q, H, W):
    B, C = gp.shape[:2]
    full = torch.zeros(B, C, H // 2, W // 2, 4, dtype=gp.dtype)
    full.scatter_(-1, q.unsqueeze(-1), gp.unsqueeze(-1))
    return full.view(B, C, H // 2, W // 2, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H, W)


FLIP_RATE_BOUND = 1e-5  # rounding-tie decision flips per decision against fp64 (tests, smoke)


def flip_bound(decisions: int, rate: float = FLIP_RATE_BOUND) -> float:
    """Largest flip count a correct fp32 kernel may show on a block of ``decisions`` units: the
    expected rounding ties ``rate * n`` (an fp32 F(4x4) conv has ~1e-5 relative error, so about
    that fraction of pre-activations sits within rounding of 0) plus a Poisson allowance
    (4 standard deviations + 2), so a 25k-unit block may show its one or two ties while a
    systematic mis-decision — hundreds of flips per 100k units — cannot hide."""
    mu = rate * decisions
    return mu + 4.0 * mu ** 0.5 + 2.0


def flip_violations(flips: dict, totals: dict, rate: float = FLIP_RATE_BOUND) -> dict:
    """Blocks whose engine-vs-fp64 decision flips exceed :func:`flip_bound`: {block: (flips,
    decisions)}. A kernel that systematically mis-decides values near 0 (sign of zero, denormal
    flush, ``>=`` for ``>``) passes the mask-conditioned score check — it compares arithmetic
    given the engine's own decisions — but not this bound."""
    return {b: (flips[b], totals[b]) for b in flips if flips[b] > flip_bound(totals[b], rate)}


@torch.no_grad()
def engine_scores_fp64(engine, x, y, conditioned=True, mode="taylor", totals=None):
    """Per-sample scores {block: (B, C_real) fp64} of one batch: ``mode="taylor"`` the signed
    sum_hw -(dL/da * a), ``"sensitivity"`` sum_hw |dL/da| (a = the block activation's output),
    with L the batch-mean cross-entropy. Returns (scores, flips): ``flips[block]`` counts the
    units whose ReLU mask or pool argmax differs between the engine and fp64 given the same
    upstream decisions (both are computed; ``conditioned`` picks which decisions the returned
    scores use and feed downstream). ``totals`` (a dict, optional) receives each block's number
    of decisions (units of its activation), the denominator of :func:`flip_violations`."""
    plan = engine.plan
    saved = engine.forward(x)[1]
    acts_f = saved["acts"]
    lin_f = saved["lin_acts"]
    h = x.double().cpu()
    B = h.shape[0]
    flips = {}
    convs = []  # per conv block: (act (pooled) NCHW, q or None, mask at act's resolution, scale, H, W)
    for i, blk in enumerate(plan.convs):
        c = blk.conv.out_channels
        scale, shift = _affine(blk)
        pre = F.conv2d(h, blk.conv.weight.detach().double().cpu(), None, padding=1)
        pre = pre * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)
        H, W = pre.shape[2:]
        hf = _nchw(acts_f[i][0], c)
        if blk.pool is not None:
            win = _windows(pre)
            q_own = win.argmax(-1)
            v_own = win.gather(-1, q_own.unsqueeze(-1)).squeeze(-1)
            m_own = v_own > 0
            q_f = acts_f[i][1].permute(0, 3, 1, 2)[:, :c].long().cpu().contiguous()
            m_f = hf > 0
            flips[i] = int(((m_f != m_own) | ((q_f != q_own) & (m_f | m_own))).sum())
            if totals is not None:
                totals[i] = int(m_f.numel())
            q, m = (q_f, m_f) if conditioned else (q_own, m_own)
            act = torch.where(m, win.gather(-1, q.unsqueeze(-1)).squeeze(-1), torch.zeros((), dtype=pre.dtype))
        else:
            m_own = pre > 0
            m_f = hf > 0
            flips[i] = int((m_f != m_own).sum())
            if totals is not None:
                totals[i] = int(m_f.numel())
            q, m = None, (m_f if conditioned else m_own)
            act = torch.where(m, pre, torch.zeros((), dtype=pre.dtype))
        convs.append((act, q, m, scale, H, W))
        h = act
    nconv = len(plan.convs)
    lin_in = [h.reshape(B, -1) if nconv else x.double().cpu().reshape(B, -1)]
    lmask = {}  # linear index -> ReLU mask (no entry: no activation, identity in the backward)
    for j, lb in enumerate(plan.linears):
        w = lb.linear.weight.detach().double().cpu()
        b = lb.linear.bias.detach().double().cpu() if lb.linear.bias is not None else 0.0
        z = lin_in[-1] @ w.t() + b
        if lb.relu is not None:
            n = lb.linear.out_features
            m_f = lin_f[j + 1].reshape(B, -1)[:, :n].cpu() > 0
            m_own = z > 0
            flips[nconv + j] = int((m_f != m_own).sum())
            if totals is not None:
                totals[nconv + j] = int(m_f.numel())
            m = m_f if conditioned else m_own
            z = torch.where(m, z, z * lb.slope)
            lmask[j] = m
        lin_in.append(z)
    logits = lin_in[-1]
    g = (torch.softmax(logits, 1) - F.one_hot(y.cpu(), logits.shape[1]).double()) / B

    def score(ga, a):
        return (ga.abs() if mode == "sensitivity" else -(ga * a)).reshape(B, a.shape[1], -1).sum(-1)

    scores = {}
    nlin = len(plan.linears)
    g_out = None
    for j in range(nlin - 1, -1, -1):
        ga = g @ plan.linears[j].linear.weight.detach().double().cpu()
        if j > 0:
            scores[nconv + j - 1] = score(ga, lin_in[j])
            m = lmask.get(j - 1)
            g = ga if m is None else torch.where(m, ga, ga * plan.linears[j - 1].slope)
        elif nconv:
            act = convs[-1][0]
            g_out = ga.view(act.shape)
    for ci in range(nconv - 1, -1, -1):
        act, q, m, scale, H, W = convs[ci]
        scores[ci] = score(g_out, act)
        if ci == 0:
            break
        gm = torch.where(m, g_out, torch.zeros((), dtype=g_out.dtype))
        g_full = _unpool(gm, q, H, W) if q is not None else gm
        g_pre = g_full * scale.view(1, -1, 1, 1)
        prev = convs[ci - 1][0]
        g_out = torch.nn.grad.conv2d_input(prev.shape, plan.convs[ci].conv.weight.detach().double().cpu(), g_pre,
                                           padding=1)
    return scores, flips
