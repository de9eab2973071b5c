"""Forward engine for ResNets (BasicBlock / Bottleneck, torchvision layout) on the HIP kernels.

BASELINE config #3 scores every bottleneck conv of a ResNet-50 with APoZ: a forward-only pass
whose per-(sample, channel) statistic is the count of positive outputs of each block's BN (the
evaluation module ``find_best_module_for_attributions`` picks for conv1/conv2, reference
graph.py:9-34, apoz.py:28-39). The generic path runs MIOpen convolutions plus one HIP channel
reduction per module; this engine runs the whole network on our own kernels instead:

  stem   NCHW -> NHWC pad to 4 channels, 7x7/2 implicit GEMM (8 taps x 4 channels per K
         slice) with the eval-mode BN folded into the epilogue affine + ReLU; 3x3/2 max-pool
  block  1x1 -> 3x3 (stride s) -> 1x1 implicit-GEMM convs (``tpamd.conv_gen``), BN folded, the
         residual add (identity or the 1x1/s downsample conv) and the final ReLU fused into the
         last conv's epilogue; APoZ counts of the block's bn1/bn2 outputs are produced by the
         conv epilogues (exact integer counts, order independent -> deterministic)
  head   global average pool + fc GEMM

fp32 throughout (exact fp32 MFMA). Works for any input size / batch; weights are re-packed
whenever a parameter changes (pruning, training).
"""
from __future__ import annotations

import weakref
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from . import epochs
from .fused_chain import CFG_RED as _RED
from .fused_chain import (_CU, _W4_SPLITS, CFG_SB, TUNER, WINO, WINO4S, WINO_LDS, _wino_splits, cpad, logits_grad,
                          sk_candidates, taylor_slots, winograd_weights)

_W4_SIZES = (56, 28, 14, 7, 32, 16, 8, 4)  # square maps of the F(4x4) kernel (band geometry for the first four)


def wino4_cands(B: int, S: int, K: int, C: int):
    """F(4x4,3x3) split-points candidates (WINO4S, channel splits) for a stride-1 pad-1 3x3 conv on
    S x S maps (wino4.hip; ResNet's 56/28/14/7-pixel maps use its band geometry: whole 4-pixel tile
    rows per block, counted across images); empty when the kernel does not apply."""
    if S not in _W4_SIZES or C % 8 or K % 32:
        return []
    tpr = (S + 3) // 4
    if S in (56, 28, 14, 7):
        br = 32 // tpr
        blocks = -(-B * tpr // br) * (K // 32)
    else:
        blocks = -(-B * tpr * tpr // 32) * (K // 32)
    sp, chunks = 1, C // 8
    while _W4_SPLITS and blocks * sp < 2 * _CU and sp * 2 <= chunks // 4 and sp < 16:
        sp *= 2
    return [(WINO4S, 1)] + ([(WINO4S, sp)] if sp > 1 else [])


@dataclass
class _Conv:
    conv: nn.Conv2d
    bn: Optional[nn.BatchNorm2d]


@dataclass
class _Block:
    convs: list            # [_Conv] in order (2 for BasicBlock, 3 for Bottleneck)
    downsample: Optional[_Conv]


@dataclass
class ResNetPlan:
    stem: _Conv
    maxpool: nn.MaxPool2d
    blocks: list = field(default_factory=list)
    fc: Optional[nn.Linear] = None


def _is_resnet(model) -> bool:
    return all(hasattr(model, a) for a in ("conv1", "bn1", "maxpool", "layer1", "layer2", "layer3", "layer4", "fc"))


def build_resnet_plan(model: nn.Module):
    """Lower a torchvision-layout ResNet, or return (None, reason)."""
    if not _is_resnet(model):
        return None, "not a torchvision-layout ResNet"
    c1 = model.conv1
    if c1.kernel_size != (7, 7) or c1.stride != (2, 2) or c1.padding != (3, 3) or c1.in_channels > 4 or c1.groups != 1:
        return None, "unsupported stem"
    mp = model.maxpool
    if not isinstance(mp, nn.MaxPool2d) or mp.ceil_mode or mp.dilation not in (1, (1, 1)):
        return None, "unsupported stem pool"
    plan = ResNetPlan(_Conv(c1, model.bn1), mp, fc=model.fc)
    for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
        for blk in layer:
            names = ["conv1", "conv2", "conv3"] if hasattr(blk, "conv3") else ["conv1", "conv2"]
            convs = []
            for i, n in enumerate(names):
                conv = getattr(blk, n)
                bn = getattr(blk, "bn" + str(i + 1))
                if conv.groups != 1 or conv.dilation != (1, 1) or conv.kernel_size[0] not in (1, 3) or \
                        conv.padding[0] != conv.kernel_size[0] // 2:
                    return None, f"unsupported conv {conv}"
                convs.append(_Conv(conv, bn))
            ds = None
            if blk.downsample is not None:
                d = blk.downsample
                if not (isinstance(d, nn.Sequential) and len(d) == 2 and isinstance(d[0], nn.Conv2d)
                        and isinstance(d[1], nn.BatchNorm2d) and d[0].kernel_size == (1, 1)):
                    return None, "unsupported downsample"
                ds = _Conv(d[0], d[1])
            plan.blocks.append(_Block(convs, ds))
    return plan, ""


def _fold(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d]):
    w = conv.weight.detach().float()
    cout = w.shape[0]
    bias = conv.bias.detach().float() if conv.bias is not None else torch.zeros(cout, device=w.device)
    if bn is None:
        return torch.ones(cout, device=w.device), bias
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    g = bn.weight.float() if bn.weight is not None else torch.ones_like(inv)
    beta = bn.bias.float() if bn.bias is not None else torch.zeros_like(inv)
    scale = g * inv
    return scale.contiguous(), ((bias - bn.running_mean.float()) * scale + beta).contiguous()


class ResNetEngine:
    def __init__(self, model: nn.Module, plan: ResNetPlan):
        self.plan = plan
        self._key = None
        self._packed = None
        self._arena_sizes = {}  # grad_scores call shape -> floats of Taylor partial slabs it needs

    def max_batch(self, sample_shape) -> int:
        """Largest batch whose activations stay inside the kernels' 32-bit buffer descriptors
        (every tensor < 2^31 bytes) for (C, H, W) inputs; attributions/base.py runs larger
        batches in slices."""
        def out_hw(conv, H, W):
            k, s_, pd = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            return (H + 2 * pd - k) // s_ + 1, (W + 2 * pd - k) // s_ + 1

        H, W = tuple(sample_shape)[-2:]
        per = 4 * H * W * 8  # the channel-padded NHWC input
        H, W = out_hw(self.plan.stem.conv, H, W)
        per = max(per, 4 * H * W * cpad(self.plan.stem.conv.out_channels))
        mp = self.plan.maxpool
        k, s_, pd = (mp.kernel_size if isinstance(mp.kernel_size, int) else mp.kernel_size[0],
                     mp.stride if isinstance(mp.stride, int) else mp.stride[0],
                     mp.padding if isinstance(mp.padding, int) else mp.padding[0])
        H, W = (H + 2 * pd - k) // s_ + 1, (W + 2 * pd - k) // s_ + 1
        for b in self.plan.blocks:
            h, w = H, W
            for c in b.convs:
                h, w = out_hw(c.conv, h, w)
                per = max(per, 4 * h * w * cpad(c.conv.out_channels))
            H, W = h, w
        return max(1, ((1 << 31) - 1) // per)

    def _all_convs(self):
        p = self.plan
        out = [p.stem]
        for b in p.blocks:
            out += b.convs + ([b.downsample] if b.downsample is not None else [])
        return out

    def _params_key(self):
        key = []
        for c in self._all_convs():
            for t in (c.conv.weight, c.conv.bias) + ((c.bn.weight, c.bn.bias, c.bn.running_mean, c.bn.running_var)
                                                     if c.bn is not None else ()):
                if t is not None:
                    key.append((t.data_ptr(), t._version, tuple(t.shape)))
        for t in (self.plan.fc.weight, self.plan.fc.bias):
            if t is not None:
                key.append((t.data_ptr(), t._version, tuple(t.shape)))
        key.append(epochs.engine_key())  # fused optimizers / native BN stats leave versions alone
        return tuple(key)

    @torch.no_grad()
    def _pack_conv(self, c: _Conv, stem=False):
        w = c.conv.weight.detach().float()
        cout = w.shape[0]
        # activations carry channels zero-padded to a multiple of 32 (pruned, odd widths):
        # padded filters have zero weights and a zero affine -> exact zeros downstream
        cin_p = 4 if stem else cpad(w.shape[1])
        w = F.pad(w, (0, 0, 0, 0, 0, cin_p - w.shape[1], 0, cpad(cout) - cout))
        wk = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        k_pad = ops.require().conv_gen_k(c.conv.kernel_size[0], w.shape[1]) - wk.shape[1]
        if k_pad:
            wk = F.pad(wk, (0, k_pad))
        scale, shift = _fold(c.conv, c.bn)
        scale, shift = F.pad(scale, (0, cpad(cout) - cout)), F.pad(shift, (0, cpad(cout) - cout))
        e = {"w": wk.contiguous(), "scale": scale, "shift": shift, "ks": c.conv.kernel_size[0],
             "stride": c.conv.stride[0], "pad": c.conv.padding[0]}
        if e["ks"] == 3 and e["stride"] == 1 and w.shape[1] % 8 == 0 and w.shape[0] % 32 == 0:
            e["u"] = winograd_weights(w)  # stride-1 3x3: Winograd candidate
            e["w4d"] = w.contiguous()     # F(4x4) U images built on first use (_u4)
        return e

    def _pack(self):
        key = self._params_key()
        if key == self._key:
            return self._packed
        p = self.plan
        blocks = []
        for b in p.blocks:
            blocks.append({"convs": [self._pack_conv(c) for c in b.convs],
                           "ds": self._pack_conv(b.downsample) if b.downsample is not None else None})
        fc_w = p.fc.weight.detach().float()
        fc_w = F.pad(fc_w, (0, cpad(fc_w.shape[1]) - fc_w.shape[1]))
        fc_b = p.fc.bias.detach().float() if p.fc.bias is not None else torch.zeros(fc_w.shape[0],
                                                                                   device=fc_w.device)
        n_cls = fc_w.shape[0]
        # fc backward operand for the MFMA GEMM: (C, classes padded to 32) with zero columns
        fc_wt = F.pad(fc_w, (0, 0, 0, cpad(n_cls) - n_cls)).t().contiguous()
        self._packed = {"stem": self._pack_conv(p.stem, stem=True), "blocks": blocks,
                        "fc_w": fc_w.contiguous(), "fc_b": fc_b.contiguous(), "fc_wt": fc_wt}
        self._key = key
        return self._packed

    @staticmethod
    def _u4(T, e, dgrad=False):
        """F(4x4) U images of a stride-1 3x3 conv (forward, or the data gradient's flipped /
        transposed operand with the BN scale folded in), cached in the packed entry."""
        key = "ut4" if dgrad else "u4"
        if key not in e:
            e[key] = T.wino4_weights(e["w4t"] if dgrad else e["w4d"], dgrad, 0, 0)
        return e[key]

    @staticmethod
    def _conv(T, e, h, relu, res=None, apoz=None):
        B, H, W, C = h.shape
        ks, s, pd = e["ks"], e["stride"], e["pad"]
        Ho, Wo = (H + 2 * pd - ks) // s + 1, (W + 2 * pd - ks) // s + 1
        M, N, K = B * Ho * Wo, e["scale"].numel(), e["w"].shape[1]
        cands = TUNER.candidates(M, N, K)
        if C != 4:
            cands = cands + sk_candidates(T, cands, ks, M, N)
            if ks == 1 and K <= 256:  # short K: the single-buffered LDS stage (twice the blocks per CU)
                cands = cands + [(CFG_SB | c, 1) for c in (2, 3, 6)]
        if "u" in e and res is None:  # odd H / W: partial last tile row / column (direct loads)
            sp0 = _wino_splits(B * ((H + 1) // 2) * ((W + 1) // 2), N, C)
            cands = [(WINO_LDS, sp0), (WINO, sp0)] + ([(WINO_LDS, 1)] if sp0 > 1 else []) + cands
            if H == W and pd == 1:
                cands = cands + wino4_cands(B, H, N, C)
        key = ("gen", tuple(h.shape), N, ks, s, res is not None)

        def run(cfg, sp, hh=h, ap=None):
            if cfg in (WINO, WINO_LDS):
                return T.conv_wino_fwd(hh, e["u"], e["scale"], e["shift"], relu, False, sp, cfg == WINO_LDS, ap)[0]
            if cfg == WINO4S:
                return T.conv_wino4_fwd(hh, ResNetEngine._u4(T, e), e["scale"], e["shift"], relu, False, ap, sp, 3)[0]
            return T.conv_gen(hh, e["w"], e["scale"], e["shift"], relu, res, ap, ks, s, pd, cfg, sp)

        cfg, sp = TUNER.choose(key, M, N, K, run, cands=cands)
        return run(cfg, sp, h, apoz)

    def forward(self, x: torch.Tensor, apoz: Optional[dict] = None, save: bool = False):
        """Logits of the network; ``apoz`` maps BN modules of the blocks (bn1 / bn2 / ...) to
        zeroed (B, C) float tensors that receive the per-sample counts of positive outputs.
        ``save=True`` returns (logits, saved) with, per block, (input, internal post-ReLU
        activations, output) in engine layout (NHWC, channel-padded) for :meth:`grad_scores`."""
        T = ops.require()
        P = self._pack()
        apoz = dict(apoz or {})
        padded = []  # (user buffer, padded scratch) for channel counts that are not multiples of 32
        for m, buf in apoz.items():
            if buf.shape[1] % 32:
                tmp = buf.new_zeros(buf.shape[0], cpad(buf.shape[1]))
                padded.append((buf, tmp))
                apoz[m] = tmp
        h = self._stem(T, P, x, apoz)
        saved = []
        for blk, e in zip(self.plan.blocks, P["blocks"]):
            h = self._block(T, blk, e, h, apoz, saved if save else None)
        feat = T.avgpool_nhwc(h)
        for buf, tmp in padded:
            buf.add_(tmp[:, :buf.shape[1]])
        logits = self._fc(T, P, feat)
        if save:
            saved.append(feat)
            return logits, saved
        return logits

    @staticmethod
    def _fc(T, P, feat):
        """Classifier GEMM on the MFMA kernel (ks=1 implicit GEMM, bias in the epilogue)."""
        B, C = feat.shape
        w = P["fc_w"]
        x = feat.contiguous().view(B, 1, 1, C)
        cfg, sp = TUNER.choose(("fc", B, C, w.shape[0]), B, w.shape[0], C,
                               lambda c, s_: T.conv_fwd(x, w, None, P["fc_b"], False, False, 1, c, s_))
        return T.conv_fwd(x, w, None, P["fc_b"], False, False, 1, cfg, sp)[0].view(B, -1)

    @staticmethod
    def _fc_bwd(T, P, g_log, feat):
        """dL/dfeat = g_log @ fc_w on the MFMA kernel (classes zero-padded to 32; the epilogue's
        ReLU mask by feat > 0 is exact here: feat is an average of ReLU outputs, and a zero
        average means every pixel of that channel is 0, masked again downstream)."""
        B, C = feat.shape
        wt = P["fc_wt"]
        g = F.pad(g_log, (0, wt.shape[1] - g_log.shape[1])).contiguous().view(B, 1, 1, -1)
        a = feat.contiguous().view(B, 1, 1, C)
        cfg, sp = TUNER.choose(("fc_bwd", B, C, wt.shape[1]), B, C, wt.shape[1],
                               lambda c, s_: T.conv_dgrad(g, None, wt, a, None, None, True, 1, c, s_))
        return T.conv_dgrad(g, None, wt, a, None, None, True, 1, cfg, sp).view(B, C)

    def _stem(self, T, P, x, apoz):
        h = T.nchw_to_nhwc_pad(x.float().contiguous(), 4)
        h = self._conv(T, P["stem"], h, True, apoz=apoz.get(self.plan.stem.bn))
        mp = self.plan.maxpool
        k = mp.kernel_size if isinstance(mp.kernel_size, int) else mp.kernel_size[0]
        s = mp.stride if isinstance(mp.stride, int) else mp.stride[0]
        pd = mp.padding if isinstance(mp.padding, int) else mp.padding[0]
        return T.maxpool_nhwc(h, k, s, pd)

    def _block(self, T, blk, e, h, apoz=None, saved=None):
        """One residual block: downsample / identity, convs with the residual add + ReLU fused
        into the last conv's epilogue; appends (input, inner activations, output) to ``saved``."""
        apoz = apoz or {}
        idn = self._conv(T, e["ds"], h, False) if e["ds"] is not None else h
        t = h
        n = len(e["convs"])
        inner = []
        for i, (c, ce) in enumerate(zip(blk.convs, e["convs"])):
            last = i == n - 1
            t = self._conv(T, ce, t, True, res=idn if last else None, apoz=apoz.get(c.bn))
            if not last:
                inner.append(t)
        if saved is not None:
            saved.append((h, inner, t))
        return t

    # ------------------------------------------------------------------ partial forward (Shapley)
    def locate(self, bn):
        """(block, conv) index whose BN output ``bn`` is, for the block-internal BNs."""
        for bi, blk in enumerate(self.plan.blocks):
            for ci, c in enumerate(blk.convs[:-1]):
                if c.bn is bn:
                    return bi, ci
        raise KeyError("not a block-internal BatchNorm of this ResNet")

    def forward_to(self, x: torch.Tensor, bi: int, ci: int):
        """(post-ReLU output of conv ``ci`` of block ``bi``, that block's residual operand), both
        in engine layout: the state ``logits_from`` continues from. Masking a channel of the BN
        output equals masking it after the ReLU (ReLU(0) = 0)."""
        T = ops.require()
        P = self._pack()
        h = self._stem(T, P, x, {})
        for b in range(bi):
            h = self._block(T, self.plan.blocks[b], P["blocks"][b], h)
        e = P["blocks"][bi]
        idn = self._conv(T, e["ds"], h, False) if e["ds"] is not None else h
        t = h
        for i in range(ci + 1):
            t = self._conv(T, e["convs"][i], t, True)
        return t, idn

    def logits_from(self, bi: int, ci: int, a: torch.Tensor, idn: torch.Tensor) -> torch.Tensor:
        """Logits of the network continued from ``forward_to``'s state (``a`` possibly masked and
        stacked K times along the batch, ``idn`` stacked the same way)."""
        T = ops.require()
        P = self._pack()
        e = P["blocks"][bi]
        n = len(e["convs"])
        t = a
        for i in range(ci + 1, n):
            t = self._conv(T, e["convs"][i], t, True, res=idn if i == n - 1 else None)
        for b in range(bi + 1, len(self.plan.blocks)):
            t = self._block(T, self.plan.blocks[b], P["blocks"][b], t)
        return self._fc(T, P, T.avgpool_nhwc(t))

    # ------------------------------------------------------------------ backward (Taylor, Sensitivity)
    @staticmethod
    @torch.no_grad()
    def _bwd_operands(e):
        """dgrad operands of a packed conv, cached in its entry: the BN scale of the conv's
        output is folded into the weights' output channels (the gradient leaving a masked
        epilogue is dL/d(BN output); the next GEMM consumes dL/d(conv output) = that x scale)."""
        if "wt" in e:
            return e
        ks = e["ks"]
        co = e["scale"].numel()
        ci = e["w"].shape[1] // (ks * ks)
        w4 = e["w"].view(co, ks, ks, ci) * e["scale"].view(co, 1, 1, 1)  # (co, kh, kw, ci)
        if ks == 1:
            e["wt"] = w4.view(co, ci).t().contiguous()
        elif e["stride"] == 1:  # stride-1 3x3 dgrad = conv of g with flipped taps
            e["wt"] = w4.flip(1, 2).permute(3, 1, 2, 0).reshape(ci, ks * ks * co).contiguous()
            e["ut"] = winograd_weights(w4.permute(0, 3, 1, 2).flip(2, 3).transpose(0, 1))
            e["w4t"] = w4.permute(0, 3, 1, 2).contiguous()  # (co, ci, 3, 3): wino4_weights flips it
        else:  # strided: transposed gather kernel, natural tap order
            e["wt"] = w4.permute(3, 1, 2, 0).reshape(ci, ks * ks * co).contiguous()
        return e

    @staticmethod
    def _slab(arena, R, B, N, dev):
        """A zeroed (R, B, N) Taylor partial slab: a view into this call's arena (one zero-fill
        for every layer instead of one per layer) when it fits, else its own allocation. The
        arena records what the call asked for, so the next call of the same shape gets one that
        fits (views start on 256-B boundaries)."""
        n = R * B * N
        if arena is None:
            return torch.zeros(R, B, N, device=dev)
        arena[2] += (n + 63) // 64 * 64
        buf, off = arena[0], arena[1]
        if buf is not None and off + n <= buf.numel():
            arena[1] = off + (n + 63) // 64 * 64
            return buf[off:off + n].view(R, B, N)
        return torch.zeros(R, B, N, device=dev)

    def _dgrad(self, T, e, g, mask, res=None, res_stride=1, low_res=False, tay_mode=None, arena=None):
        """dL/d(input) of conv ``e`` from g = dL/d(conv output) (BN scale folded in), plus
        ``res``, masked by ``mask`` (the input's post-ReLU activation). ``low_res``: a strided
        1x1 conv's gradient at the output resolution (scattered by the consumer's res_stride).
        Returns (gradient, partial slab or None): with ``tay_mode`` 0, a Winograd 3x3 dgrad, a
        1x1 dgrad (implicit GEMM, one K pass) or a strided 3x3 one (transposed implicit GEMM,
        even output size: one slot range per stride phase) also writes the per-(image, channel) partial sums of
        -(dL/da * a), a = ``mask``, into an (R, B, C) slab from its epilogue (one writer per
        element: deterministic), which saves the separate channel reduction's read of both
        tensors; ``tay_mode`` 1 (Sensitivity): sums of |dL/da| of the masked gradient (the
        Winograd epilogue masks it by a > 0 itself: its tay_mode 2)."""
        e = self._bwd_operands(e)
        B, H, W, C = g.shape
        ks, s = e["ks"], e["stride"]
        N = e["wt"].shape[0]
        transposed = s > 1 and not low_res
        Ho, Wo = (mask.shape[1], mask.shape[2]) if transposed else (H, W)
        M, K = B * Ho * Wo, e["wt"].shape[1]
        pad = e["pad"] if (transposed or ks == 3) else 0
        if transposed:
            cands = [(c, 1) for c in (0, 3, 4, 1, 5, 6, 2)]
        else:
            cands = TUNER.candidates(M, N, K)
            cands = cands + sk_candidates(T, cands, ks, M, N, tay=False)
            if ks == 1 and K <= 256:
                cands = cands + [(CFG_SB | c, 1) for c in (2, 3, 6)]
        wino_ok = "ut" in e and res is None and mask is not None
        if wino_ok:
            sp0 = _wino_splits(B * ((H + 1) // 2) * ((W + 1) // 2), N, C)
            cands = [(WINO_LDS, sp0), (WINO, sp0)] + cands
            if H == W and e["pad"] == 1:
                cands = cands + wino4_cands(B, H, N, C)
        key = ("rbwd", tuple(g.shape), N, ks, s, transposed, res is not None, res_stride, mask is not None)

        # implicit-GEMM dgrads with fused Taylor partials: 1x1 (one K pass, tiles spanning <= 4
        # images), and the strided 3x3 ones (parity row order: <= 4 (phase, image) row groups)
        gen_tay = tay_mode is not None and mask is not None and res is None and (
            (ks == 1 and not transposed) or (transposed and ks == 3 and s == 2 and Ho % 2 == 0 and Wo % 2 == 0))

        def tay_slots(c):
            return 4 * T.conv_gen_tay_slots(c, Ho * Wo // 4) if transposed else T.conv_gen_tay_slots(c, Ho * Wo)
        if gen_tay:
            # the tuner weighs each fused-partials config against every plain config followed by
            # the separate channel reduction (tuner-only flag _RED): the configs that cannot carry
            # the partials' registers are sometimes the fastest tiles
            plain = list(dict.fromkeys((c, 1) for c, _ in cands if c >= 0))
            tay_c = [(c, 1) for c, _ in plain if tay_slots(c) > 0]
            gen_tay = bool(tay_c)
            if gen_tay:
                cands = tay_c + [(c | _RED, 1) for c, _ in plain]
                key = key + ("tay",)

        def run(cfg, sp, gg=g, rr=res, mm=mask, tay=None):
            if cfg in (WINO, WINO_LDS):  # Sensitivity of the BN before the ReLU: |g| where a > 0 (mode 2)
                return T.conv_wino_dgrad(gg, None, e["ut"], mm, None, tay, True, sp, cfg == WINO_LDS,
                                         2 if tay_mode == 1 else 0)
            if cfg == WINO4S:
                return T.conv_wino4_dgrad(gg, ResNetEngine._u4(T, e, True), mm, None, tay, True,
                                          2 if tay_mode == 1 else 0, sp, 3)
            return T.conv_gen_bwd(gg, e["wt"], rr, res_stride, mm, ks, s if transposed else 1, pad, Ho, Wo,
                                  transposed, cfg, sp, tay, tay_mode or 0)

        def run_tay(cfg, sp):  # the tuner's view of a gen_tay candidate: kernel + partials or + reduction
            if cfg & _RED:
                o = run(cfg & ~_RED, sp)
                ops.channel_reduce(mask.permute(0, 3, 1, 2), o.permute(0, 3, 1, 2),
                                   "sensitivity" if tay_mode == 1 else "taylor")
                return o
            return run(cfg, sp, tay=torch.zeros(tay_slots(cfg), B, N, device=g.device))

        cfg, sp = TUNER.choose(key, M, N, K, run_tay if gen_tay else run, cands=cands if cands else None)
        if gen_tay and cfg & _RED:  # plain kernel: grad_scores runs the channel reduction
            return run(cfg & ~_RED, sp), None
        if tay_mode is not None and cfg in (WINO, WINO_LDS):
            tay = self._slab(arena, taylor_slots(Ho, Wo), B, N, g.device)
            return run(cfg, sp, tay=tay), tay
        if tay_mode is not None and cfg == WINO4S:
            tay = self._slab(arena, T.wino4_taylor_slots(Ho), B, N, g.device)
            return run(cfg, sp, tay=tay), tay
        if gen_tay:
            tay = self._slab(arena, tay_slots(cfg), B, N, g.device)
            return run(cfg, sp, tay=tay), tay
        return run(cfg, sp), None

    def grad_scores(self, x: torch.Tensor, y: torch.Tensor, want, mode: str, criterion=None,
                    loss_batch: Optional[int] = None, raw_slabs: bool = False):
        """One engine forward + input-gradient-only backward of the loss (mean cross-entropy on
        the fused kernel, or ``criterion`` through autograd on the logits); returns
        {BN module: (B, C_padded) per-sample ``ops.channel_reduce`` score} for the block BNs in
        ``want`` (evaluation modules of conv1/conv2 of each block). No weight gradients, no
        autograd graph; the backward stops at the earliest block holding a wanted BN.
        ``raw_slabs``: a score that came from a data-gradient epilogue stays its raw (R, B, C_padded)
        partial-slot slab (no slot sum, no |.|) for ``ops.score_fold_`` to finish in its single
        launch (take_abs for "taylor"; |.| of the other, already final slabs changes nothing)."""
        T = ops.require()
        P = self._pack()
        logits, saved = self.forward(x, save=True)
        feat = saved.pop()
        B = logits.shape[0]
        g_log = logits_grad(logits, y, criterion, loss_batch)
        g_feat = self._fc_bwd(T, P, g_log, feat)  # (B, C_last padded)
        y_last = saved[-1][2]
        HW = y_last.shape[1] * y_last.shape[2]
        # avg-pool backward + final ReLU of the last block: dL/d(pre-ReLU residual sum)
        g_s = torch.where(y_last > 0, (g_feat / HW)[:, None, None, :], torch.zeros((), device=x.device)).contiguous()
        blocks = self.plan.blocks
        first = min((bi for bi, b in enumerate(blocks) if any(c.bn in want for c in b.convs[:-1])), default=None)
        out = {}
        if first is None:
            return out
        # one zero-filled arena for the call's Taylor partial slabs: [buffer, offset, floats asked]
        akey = (tuple(x.shape), mode, tuple(sorted(i for i, m in enumerate(self.eval_modules()) if m in want)))
        size = self._arena_sizes.get(akey)
        arena = [torch.zeros(size, device=x.device) if size else None, 0, 0]
        for bi in range(len(blocks) - 1, first - 1, -1):
            blk, e = blocks[bi], P["blocks"][bi]
            x_in, inner, _ = saved[bi]
            g = g_s
            for ci in range(len(blk.convs) - 1, 0, -1):
                a_prev = inner[ci - 1]
                bn = blk.convs[ci - 1].bn
                tm = ({"taylor": 0, "taylor_signed": 0, "sensitivity": 1}.get(mode) if bn in want else None)
                g, tay = self._dgrad(T, e["convs"][ci], g, a_prev, tay_mode=tm,
                                     arena=arena)  # dL/d(bn_{ci} output), masked
                if tay is not None:  # partials from the data-gradient epilogue
                    if raw_slabs:
                        out[bn] = tay
                    else:
                        sums = tay.sum(0)
                        out[bn] = sums.abs_() if mode == "taylor" else sums
                elif bn in want:
                    out[bn] = ops.channel_reduce(a_prev.permute(0, 3, 1, 2), g.permute(0, 3, 1, 2), mode)
            if bi == first:
                break
            if e["ds"] is not None:
                g_res, _ = self._dgrad(T, e["ds"], g_s, None, low_res=True)
                rs = e["ds"]["stride"]
            else:
                g_res, rs = g_s, 1
            g_s, _ = self._dgrad(T, e["convs"][0], g, x_in, res=g_res, res_stride=rs)
        if arena[2] > (size or 0):
            self._arena_sizes[akey] = arena[2]
        return out

    def eval_modules(self):
        """BN modules whose outputs the engine can count (block bn1/bn2/..., stem bn)."""
        mods = [self.plan.stem.bn]
        for b in self.plan.blocks:
            mods += [c.bn for c in b.convs[:-1]]
        return mods


_ENGINES: "weakref.WeakKeyDictionary[nn.Module, ResNetEngine]" = weakref.WeakKeyDictionary()


def maybe_resnet_engine(model, eval_modules, device, grad=False, why=None):
    """A ResNetEngine when every eval module is a BN the engine counts (``grad``: scores by
    :meth:`ResNetEngine.grad_scores`, block BNs only), else None (``why`` receives the reason)."""
    from .fused_chain import _reject, engines_enabled
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    if not engines_enabled():
        return _reject(why, "resnet engine: engines disabled (TORCHPRUNER_ENGINES=0)")
    if dev.type != "cuda" or ops.backend() == "torch" or not ops.available() or model.training:
        return _reject(why, "resnet engine: needs an eval-mode model on a GPU with the native extension")
    if any(p.dtype != torch.float32 for p in model.parameters()):
        return _reject(why, "resnet engine: parameters are not float32")
    plan, reason = build_resnet_plan(model)  # re-validated every run: pruning changes channel counts
    if plan is None:
        return _reject(why, f"resnet engine: {reason}")
    eng = _ENGINES.get(model)
    if eng is None or [c.conv for c in eng._all_convs()] != [c.conv for c in ResNetEngine(model, plan)._all_convs()]:
        eng = ResNetEngine(model, plan)
        _ENGINES[model] = eng
    ok = set(map(id, eng.eval_modules()[1:] if grad else eng.eval_modules()))
    if not all(id(m) in ok for m in eval_modules):
        return _reject(why, "resnet engine: evaluation modules must be block BatchNorms "
                            "(use find_best_evaluation_module=True)")
    return eng
