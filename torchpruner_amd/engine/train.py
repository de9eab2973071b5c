"""Native convolutions for training: the finetune half of prune -> finetune (BASELINE config #5),
and the convolutions of the generic attribution path (any model with standard convs).

The reference finetunes with cuDNN convolutions (experiments/utils/train.py:11-48). On ROCm the
library path is MIOpen, which JIT-compiles and benchmarks kernels for every new convolution
shape: after each pruning round every pruned layer has a new shape, and the first steps of the
round pay 20-40 s of compilation (profiles/archive/resnet50_prune_finetune_1gpu.log). Here the
convolutions of a model run on the precompiled gfx950 kernels instead, through autograd:

  forward   implicit-GEMM fp32 MFMA conv (``tpamd.conv_gen``), bias in the epilogue
  dgrad     stride 1: the same kernel on flipped, transposed weights; strided: the transposed
            gather kernel with parity-ordered rows (``tpamd.conv_gen_bwd``)
  wgrad     pixel-split MFMA GEMM, deterministic split combine (``tpamd.conv_wgrad``, K3); for
            stride-1 3x3 also Winograd F(2x2,3x3) (``tpamd.wino_wgrad``: 16 batched GEMMs over the
            transformed tiles, 2.25x fewer multiplies), picked per shape by the tuner

Training-mode ``BatchNorm2d`` runs on deterministic NHWC batch-statistics / normalisation /
backward kernels (K5, ``tpamd.bn_train_*``), training-mode ``nn.Dropout`` on a counter-based
Philox kernel (K7b, mask regenerated in the backward), max-pool (argmax byte + gather backward)
and global average pool on NHWC kernels, ``nn.Linear`` on the MFMA GEMM; the loss and the optimizer
stay PyTorch ops (autograd composes everything), so any model works; only modules the kernels
support are switched. Pruned (odd) channel counts run unpadded in the GEMMs' K loops (a tap's last
32-wide K slice is zero-filled past the real width in the loads) and are carried between the
kernels at a granule of 8 channels (:func:`_act_w`: the F(4x4) input granule; the zero channels are
exact zeros through BN / ReLU / max-pool): inside a residual block or an ``nn.Sequential`` the
padded activation flows conv -> BN -> conv without slice / pad copies, and the training BN takes
the real width as its parameter count (``cr``). The parameters, their gradients and the
optimizer state keep the module's real shapes.
Every kernel choice is timed once per shape (``TUNER``, like ``cudnn.benchmark``) — a few
milliseconds instead of a JIT compile.
"""
from __future__ import annotations

import contextlib
import math
import os
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from . import epochs
from .fused_chain import _CU, CFG_SB, TUNER, WINO, WINO4S, WINO_LDS, _wino_splits, cpad, sk_candidates
from .resnet_engine import wino4_cands


def _wino_ok(ks, stride, pad, H, W, cin, cout) -> bool:
    """Winograd F(2x2,3x3) applies: 3x3, stride 1, "same" padding, the kernels' granules."""
    return ks == 3 and stride == 1 and pad == 1 and cin % 8 == 0 and cout % 32 == 0  # odd H / W: partial tiles


def _as_nchw(t: torch.Tensor) -> torch.Tensor:
    """(B, C, H, W) channels_last tensor on the storage of a contiguous NHWC ``t`` that is NOT an
    autograd view of it: a custom Function's output may then be modified in place
    (``ReLU(inplace=True)`` right after a BatchNorm)."""
    B, H, W, C = t.shape
    out = t.new_empty(0)
    out.set_(t.untyped_storage(), t.storage_offset(), (B, C, H, W), (H * W * C, 1, W * C, C))
    return out


def _geom(conv: nn.Conv2d):
    return conv.kernel_size[0], conv.stride[0], conv.padding[0]


def eligible(conv: nn.Module) -> bool:
    """Whether ``conv`` runs on the native kernels: square 1x1 / 3x3 / 5x5 kernels (strided 5x5
    excluded: no transposed 5x5 dgrad), any zero padding up to ks-1, or a 7x7 stem on <= 4 input
    channels; groups 1, no dilation. Tiny-Cin (<= 4) 3x3 / 5x5 / 7x7 layers use the 4-channel
    packed-tap kernel instead of padding the input to 32 channels."""
    if not isinstance(conv, nn.Conv2d) or conv.groups != 1 or conv.dilation != (1, 1):
        return False
    if conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        return False
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if k[0] != k[1] or s[0] != s[1] or p[0] != p[1] or p[0] > k[0] - 1:
        return False
    if k[0] == 7:
        return conv.in_channels <= 4
    if k[0] == 5:
        return s[0] == 1
    return k[0] in (1, 3)


def _act_w(c: int) -> int:
    """Channel width a native activation carries: the next multiple of 8 (the F(4x4) kernel's input
    granule; the implicit GEMMs take any multiple of 4, BN any width). A 20 %-pruned ResNet-50
    layer of 103 channels carries 104 (the round-5 32-granule carried 128)."""
    return -(-max(c, 8) // 8) * 8


def _r32(c: int) -> int:
    return -(-c // 32) * 32


def _cin_pad(ks: int, cin: int) -> int:
    """Input width the kernels see: 4 (packed taps) for tiny-Cin 3x3/5x5/7x7, else :func:`_act_w`."""
    return 4 if (ks in (3, 5, 7) and cin <= 4) else _act_w(cin)


def _kslice(cin_p: int) -> int:
    """Channels per tap in a GEMM weight operand: 4 (packed taps) or the 32-wide K slices."""
    return 4 if cin_p == 4 else _r32(cin_p)


def _wgrad_splits(P, tiles):
    slices = math.ceil(P / 32)
    sp = 1
    while tiles * sp < 2 * _CU and sp * 2 <= max(1, slices // 8):
        sp *= 2
    return sp


def _wgrad_wave_splits(P, tiles):
    """Split counts that fill whole waves of one or two co-resident blocks per CU: a power-of-two
    split can leave a mostly empty last wave (ResNet-50's 7-px 3x3 wgrad: 144 tiles x 4 splits =
    2.25 waves of its one-block-per-CU 128x128 kernel)."""
    slices = math.ceil(P / 32)
    out = set()
    for per_cu in (1, 2):
        for waves in (1, 2, 3, 4):
            sp = waves * per_cu * _CU // max(1, tiles)
            if 1 <= sp <= max(1, slices // 8):
                out.add(sp)
    return sorted(out)


# TORCHPRUNER_BN_EPI_STATS=0: training BN always runs its own statistics pass (A/B switch)
_EPI_STATS = os.environ.get("TORCHPRUNER_BN_EPI_STATS", "1") != "0"


# TORCHPRUNER_BATCH_WEIGHT_PACK=0: one pack launch per operand and use (A/B switch)
_BATCH_PACK = os.environ.get("TORCHPRUNER_BATCH_WEIGHT_PACK", "1") != "0"


# TORCHPRUNER_BN_BWD_FUSE=0: a bottleneck's backward keeps the separate BN statistics pass and the
# materialised residual gradient (A/B switch, read once per process)
_BWD_FUSE = os.environ.get("TORCHPRUNER_BN_BWD_FUSE", "1") != "0"
# backward passes that took each fusion (tests / diagnostics): tail statistics from a dgrad epilogue,
# identity gradients handed over unmasked
FUSE_COUNTS = {"bn_stats_from_dgrad": 0, "raw_residual": 0}


class _BNLink:
    """What a training BN(+ReLU) tail (:class:`_NativeBNAct`) shares with the residual-block entry
    nodes next to it (:class:`_NativeBlockEntry`), so two of its backward passes over the block
    output can ride in conv1's data-gradient GEMM epilogue instead:

    * raw residual gradient (``raw_res``, the block's own tail, identity shortcut): the tail's
      backward hands its incoming gradient to the identity branch unmasked (no masked copy
      written); the entry's conv1 dgrad epilogue masks it by the tail's ReLU bits ``mk``;
    * backward statistics (the previous block's tail, whose output is this block's input): the
      entry's conv1 dgrad epilogue produces that tail's incoming gradient and reduces its BN
      statistics per tile (``part``); the tail's backward uses them when the gradient it receives
      is exactly that tensor, unmodified (``g_ptr`` / ``g_ver``: no other consumer added to it),
      and runs its own statistics pass otherwise."""

    __slots__ = ("xh", "mean", "invstd", "mk", "raw_res", "part", "g_ptr", "g_ver")

    def __init__(self):
        self.xh = self.mean = self.invstd = self.mk = self.part = None
        self.raw_res = False
        self.g_ptr = self.g_ver = None


class _PackSet:
    """The zero-padded GEMM operands of the fp32 conv weights (``pack_conv_weight`` modes 0-2),
    cached across uses and repacked TOGETHER by one ``pack_conv_weights_multi`` launch: the
    optimizer step updates every weight at once, so the first request after it finds all packs
    stale and one launch refreshes them all (ResNet-50: 81 pack launches per training step -> 2,
    the descriptor copy and the kernel). An entry is stale when its weight's autograd version
    counter moved (in-place ops on the parameter) or an epoch moved (:mod:`.epochs`: any
    torch.optim step — fused kernels do not bump versions —, any forward of a native-conv model). Not seen: writes
    through ``param.data`` by hand between two forwards of a submodule called directly; use
    ``TORCHPRUNER_BATCH_WEIGHT_PACK=0`` for such loops. Entries hold a reference to their weight
    (no dangling pointer) and are dropped after a whole step without a request (pruned layers)."""

    def __init__(self):
        # key -> [weight view, out, kind, cfg, (version, OPT, FWD) packed at, last generation used]
        self.entries = {}
        self.gen = 0

    def get(self, T, w, kind, cfg, out_shape):
        """kind "pack": cfg = (rows, cols, cpad, mode) of pack_conv_weight; "w4": cfg = (K, C,
        flip_t) of wino4_weights."""
        key = (kind, w.data_ptr(), tuple(w.shape), tuple(w.stride()), str(w.device), cfg)
        e = self.entries.get(key)
        now = (w._version, epochs.OPT[0], epochs.FWD[0])
        if e is not None and e[4] == now:
            e[5] = self.gen
            return e[1]
        if e is None:
            e = [w, torch.empty(out_shape, dtype=torch.float32, device=w.device), kind, cfg, None, self.gen]
            self.entries[key] = e
        else:  # the weights moved on (optimizer step / new forward): a new generation, unused entries go
            self.gen += 1
            e[5] = self.gen  # before the sweep: the requested entry is never dropped (and is repacked below)
            self.entries = {k: v for k, v in self.entries.items() if v[5] >= self.gen - 2}
        ep = (epochs.OPT[0], epochs.FWD[0])
        stale = [v for v in self.entries.values() if v[4] != (v[0]._version, *ep) and v[0].device == w.device]
        for kd, fn in (("pack", T.pack_conv_weights_multi), ("w4", T.wino4_weights_multi)):
            lst = [v for v in stale if v[2] == kd]
            if lst:
                fn([v[0] for v in lst], [v[1] for v in lst], [c for v in lst for c in v[3]])
        for v in stale:
            v[4] = (v[0]._version, *ep)
        return e[1]


_PACKS = _PackSet()


def invalidate_packs() -> int:
    """Mark every cached training-conv weight pack stale (repacked at its next use): the explicit
    hook for weight writes the staleness check cannot see (``param.data`` edits between two
    forwards of a submodule called directly). :func:`torchpruner_amd.engine.invalidate` calls it.
    Returns the number of entries marked."""
    for v in _PACKS.entries.values():
        v[4] = None
    return len(_PACKS.entries)


def _pack(T, w, rows, cols, cpad_, mode, shared):
    """Packed GEMM operand of weight ``w``; ``shared``: w is the parameter's own storage (its
    version counter tracks in-place updates) -> the batched cache, else one launch now."""
    if shared and _BATCH_PACK:
        return _PACKS.get(T, w, "pack", (rows, cols, cpad_, mode), (rows, cols))
    return T.pack_conv_weight(w.contiguous(), rows, cols, cpad_, mode)


def _u4(T, w, K, C, flip, shared):
    """F(4x4) U images of a 3x3 weight (``wino4_weights(w, flip, K, C)``), batched like _pack."""
    if shared and _BATCH_PACK:
        return _PACKS.get(T, w, "w4", (K, C, int(flip)), (C // 8, K // 32, T.wino4_u_img()))
    return T.wino4_weights(w, flip, K, C)


def _conv_fwd(x, weight, bias, ks, stride, pad, stats=False, keep=False):
    """Forward of one native conv: returns (y NHWC (B, Ho, Wo, C'), saved (xh, w32), meta, part).
    ``x`` may carry more channels than the weight (a padded activation: zeros past the real width).
    ``keep``: y keeps its carried width C' = _act_w(Cout) (zeros past Cout) for a consumer that
    takes padded activations; else C' = Cout. With ``stats``, ``part`` is the per-tile BatchNorm
    statistics of y from the GEMM epilogue ((G, 2, C') fp64, for ``bn_act(..., pre=part)``) when
    the tuned kernel is a single-pass implicit GEMM, else None."""
    T = ops.require()
    B, Cx, H, W = x.shape
    Cout, Cin = weight.shape[0], weight.shape[1]
    cin_p = _cin_pad(ks, Cx)
    cout_p = _act_w(Cout)
    k32 = _r32(cout_p)  # the Winograd kernels' output blocks (MFMA N); stores stop at cout_p
    xh = x.permute(0, 2, 3, 1)
    if cin_p != Cx:
        xh = F.pad(xh, (0, cin_p - Cx))
    xh = xh.float().contiguous()
    wd = weight.detach()
    w32 = wd if wd.dtype == torch.float32 else wd.float()  # the parameter itself for fp32 weights: no copy
    shared = w32 is wd  # (may be channels_last: the pack / transform kernels read it in place)
    kk = T.conv_gen_k(ks, cin_p)
    shift = F.pad(bias.detach().float(), (0, cout_p - Cout)).contiguous() if bias is not None else None
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    M = B * Ho * Wo

    wino = _wino_ok(ks, stride, pad, H, W, cin_p, cout_p)
    cache = {}  # padded operands, built on first use by one HIP launch each (weights change every step)

    def run(cfg, sp):
        if cfg in (WINO, WINO_LDS):  # Winograd F(2x2,3x3): 2.25x fewer multiplies
            if "u" not in cache:
                cache["u"] = T.wino_weights(w32.contiguous(), False, cout_p, cin_p)
            return T.conv_wino_fwd(xh, cache["u"], None, shift, False, False, sp, cfg == WINO_LDS)[0]
        if cfg == WINO4S:  # Winograd F(4x4,3x3): 4x fewer multiplies (band geometry on ResNet's maps)
            if "u4" not in cache:
                cache["u4"] = _u4(T, w32, k32, cin_p, False, shared)
            return T.conv_wino4_fwd(xh, cache["u4"], None, shift, False, False, None, sp, 3, cout_p)[0]
        if "wk" not in cache:  # [cout_p][(kh, kw, ci)] zero-padded GEMM operand
            cache["wk"] = _pack(T, w32, cout_p, kk, _kslice(cin_p), 0, shared)
        return T.conv_gen(xh, cache["wk"], None, shift, False, None, None, ks, stride, pad, cfg, sp)

    cands = TUNER.candidates(M, cout_p, kk)
    if cin_p != 4:
        cands = cands + sk_candidates(T, cands, ks, M, cout_p)
    if ks == 1 and cin_p != 4 and kk <= 256:  # short K: the single-buffered LDS stage (2x blocks per CU)
        cands = cands + [(CFG_SB | c, 1) for c in (2, 3, 6)]
    if wino:
        sp0 = _wino_splits(B * ((H + 1) // 2) * ((W + 1) // 2), cout_p, cin_p)
        cands = [(WINO_LDS, sp0), (WINO, sp0)] + cands
    if ks == 3 and stride == 1 and pad == 1 and H == W and cin_p != 4:
        # unpadded output widths (cout_p < k32) need one K pass: the split slabs are k32 wide
        cands = cands + [c for c in wino4_cands(B, H, k32, cin_p) if k32 == cout_p or c[1] == 1]
    cfg, sp = TUNER.choose(("tfwd", tuple(xh.shape), cout_p, ks, stride, pad), M, cout_p, kk, run, cands=cands)
    part = None
    stats_ok = (ks in (1, 3, 5) and cin_p != 4) or (ks in (3, 5, 7) and cin_p == 4)  # conv_gen_stats' shapes
    if stats and stats_ok and _EPI_STATS and cfg not in (WINO, WINO_LDS, WINO4S) and sp == 1:
        if "wk" not in cache:
            cache["wk"] = _pack(T, w32, cout_p, kk, _kslice(cin_p), 0, shared)
        y, part = T.conv_gen_stats(xh, cache["wk"], shift, ks, stride, pad, cfg)
        if cout_p != Cout and not keep:
            part = part[..., :Cout].contiguous()
    else:
        y = run(cfg, sp)
    if cout_p != Cout and not keep:
        y = y[..., :Cout].contiguous()
    meta = (ks, stride, pad, Cin, Cout, H, W, bias is not None, weight.dtype, weight.stride(), cin_p, cout_p, Cx)
    return y, (xh, w32), meta, part


def _grad_nhwc(gy, meta):
    """dL/dy (NCHW view) -> contiguous NHWC at the carried output width (a padded output's
    gradient already has it: zeros past Cout)."""
    cout_p = meta[11]
    g = gy.permute(0, 2, 3, 1).float()
    if g.shape[-1] != cout_p:
        g = F.pad(g, (0, cout_p - g.shape[-1]))
    return g.contiguous()


def _conv_dgrad_fused(g, w32, meta, res, res_stride, res_bits, link):
    """1x1 stride-1 input gradient (conv1 of a residual block) with the bottleneck fusions of
    ``conv_gen_bwd_bn``: ``res`` masked by ``res_bits`` (a raw residual gradient, see _BNLink)
    and / or the backward statistics of ``link``'s BN (the producer of this conv's input).
    Returns (dx NHWC, tile statistics or None); one-pass implicit-GEMM tiles only."""
    T = ops.require()
    ks, stride, pad, Cin, Cout, H, W, _, _, _, cin_p, cout_p = meta[:12]
    B = g.shape[0]
    shared = meta[8] == torch.float32
    M, K = B * H * W, _kslice(cout_p)
    cache = {}

    def wt():
        if "wt" not in cache:
            cache["wt"] = _pack(T, w32, cin_p, K, K, 1, shared)
        return cache["wt"]

    def run(cfg, sp):
        return T.conv_gen_bwd(g, wt(), res, res_stride, None, 1, 1, 0, H, W, False, cfg, sp)

    cands = [c for c in TUNER.candidates(M, cin_p, K) if c[0] >= 0 and c[1] == 1]
    cands = cands + sk_candidates(T, cands, 1, M, cin_p)
    if K <= 256:
        cands = cands + [(CFG_SB | c, 1) for c in (2, 3, 6)]
    key = ("tdgrad1", tuple(g.shape), cin_p, res is not None and res_stride)
    cfg, _ = TUNER.choose(key, M, cin_p, K, run, cands=cands)
    bn = link is not None and link.xh is not None
    return T.conv_gen_bwd_bn(g, wt(), res, res_stride, res_bits, link.xh if bn else None, link.mean if bn else None,
                             link.invstd if bn else None, link.mk if bn else None, cfg)


def _conv_dgrad(g, w32, meta, res=None, res_stride=1):
    """Input gradient (B, H, W, cin_p) NHWC of a native conv (ks != 7); ``res`` (optional, NHWC,
    (B, ceil(H/res_stride), ceil(W/res_stride), cin_p)) is added in the GEMM epilogue at the pixels
    with h, w % res_stride == 0 — the other branch's gradient of a tensor read twice (residual
    blocks), without a separate add pass."""
    T = ops.require()
    ks, stride, pad, Cin, Cout, H, W, _, _, _, cin_p, cout_p = meta[:12]
    B, Ho, Wo = g.shape[0], g.shape[1], g.shape[2]
    kin, n32 = _kslice(cout_p), _r32(cin_p)  # per-tap K slice width; the F(4x4) output blocks
    # stride 1: dgrad = stride-1 conv of g with flipped taps, padding ks-1-pad;
    # strided 1x1 / 3x3: transposed gather kernel, natural tap order
    transposed = stride != 1
    shared = meta[8] == torch.float32  # w32 is the parameter's own storage (see _conv_fwd)
    assert res is None or not transposed
    pad_b = pad if transposed else ks - 1 - pad
    M, K = B * H * W, ks * ks * kin
    wino = res is None and not transposed and _wino_ok(ks, 1, pad_b, Ho, Wo, cout_p, cin_p)
    cache = {}

    def run(cfg, sp):
        if cfg in (WINO, WINO_LDS):  # stride-1 3x3 dgrad = Winograd conv of g, flipped taps
            if "ut" not in cache:
                cache["ut"] = T.wino_weights(w32.contiguous(), True, cin_p, cout_p)
            return T.conv_wino_fwd(g, cache["ut"], None, None, False, False, sp, cfg == WINO_LDS)[0]
        if cfg == WINO4S:
            if "ut4" not in cache:
                cache["ut4"] = _u4(T, w32, n32, cout_p, True, shared)
            return T.conv_wino4_fwd(g, cache["ut4"], None, None, False, False, None, sp, 3, cin_p)[0]
        if "wt" not in cache:  # [ci][(kh, kw, co)], flipped for stride 1
            cache["wt"] = _pack(T, w32, cin_p, K, kin, 2 if transposed else 1, shared)
        return T.conv_gen_bwd(g, cache["wt"], res, res_stride, None, ks, stride if transposed else 1, pad_b, H, W,
                              transposed, cfg, sp)

    cands = TUNER.candidates(M, cin_p, K) if not transposed else [(c, 1) for c in (0, 3, 4, 1, 5, 6, 2)]
    if not transposed:
        cands = cands + sk_candidates(T, cands, ks, M, cin_p)
        if ks == 1 and K <= 256:  # short K: the single-buffered LDS stage
            cands = cands + [(CFG_SB | c, 1) for c in (2, 3, 6)]
    if wino:
        cands = [(WINO_LDS, _wino_splits(B * ((H + 1) // 2) * ((W + 1) // 2), cin_p, cout_p)), (WINO, 1)] + cands
    if res is None and not transposed and ks == 3 and pad_b == 1 and H == W and cin_p != 4:
        cands = cands + [c for c in wino4_cands(B, H, n32, cout_p) if n32 == cin_p or c[1] == 1]
    key = ("tdgrad", tuple(g.shape), cin_p, ks, stride, pad, res is not None and res_stride)
    cfg, sp = TUNER.choose(key, M, cin_p, K, run, cands=cands)
    return run(cfg, sp)


_WINO_WG = 16  # wgrad tuner configs >= this: the Winograd weight gradient with GEMM tile config cfg - 16


def _conv_wgrad(g, xh, meta):
    """Weight gradient in the parameter's exact shape / strides (DDP bucket views expect them),
    written by the wgrad kernel / its split combine straight from the GEMM (no re-layout copies)."""
    T = ops.require()
    ks, stride, pad, Cin, Cout, _, _, _, wdtype, w_strides, cin_p, cout_p = meta[:12]
    kk = -(-ks * ks * cin_p // 32) * 32
    P = g.shape[0] * g.shape[1] * g.shape[2]
    dw32 = torch.empty_strided((Cout, Cin, ks, ks), w_strides, dtype=torch.float32, device=g.device)

    def run_w(cfg, sp):
        if cfg >= _WINO_WG:  # Winograd F(2x2,3x3) weight gradient: 16 batched GEMMs over 2x2 tiles
            return T.wino_wgrad(g, xh, cfg - _WINO_WG, sp, dw32)
        return T.conv_wgrad(g, xh, ks, stride, pad, cfg, sp, dw32)

    cands = []
    for cfg, (bm, bn) in ((0, (128, 128)), (2, (128, 64)), (1, (64, 64))):
        tiles = math.ceil(cout_p / bm) * math.ceil(kk / bn)
        sp = _wgrad_splits(P, tiles)
        cands += [(cfg, sp)] + ([(cfg, sp // 2)] if sp > 1 else [])
        cands += [(cfg, s_) for s_ in _wgrad_wave_splits(P, tiles) if s_ not in (sp, sp // 2)]
    H, W = meta[5], meta[6]
    if ks == 3 and stride == 1 and pad == 1 and H % 2 == 0 and W % 2 == 0 and cin_p != 4:
        tiles = g.shape[0] * (H // 2) * (W // 2)
        for cfg, (bm, bn) in ((0, (128, 128)), (2, (128, 64)), (1, (64, 64))):
            sp = _wgrad_splits(tiles, 16 * math.ceil(cout_p / bm) * math.ceil(cin_p / bn))
            cands += [(_WINO_WG + cfg, sp)] + ([(_WINO_WG + cfg, sp // 2)] if sp > 1 else [])
    cfg, sp = TUNER.choose(("twgrad", tuple(g.shape), tuple(xh.shape), ks, stride, pad), cout_p, kk, P, run_w,
                           cands=cands)
    run_w(cfg, sp)
    if wdtype == torch.float32:
        return dw32
    return torch.empty_strided((Cout, Cin, ks, ks), w_strides, dtype=wdtype, device=g.device).copy_(dw32)


def _dx_nchw(dxh, meta):
    """Input gradient NHWC (B, H, W, cin_p) -> (B, Cx, H, W) for the forward's input of Cx channels
    (a channels_last view when cin_p == Cx, the carried width of a padded input)."""
    Cx = meta[12]
    if dxh.shape[-1] != Cx:
        dxh = dxh[..., :Cx]
    return dxh.permute(0, 3, 1, 2)


class _NativeConv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, ks, stride, pad, keep=False):
        y, saved, ctx.meta, _ = _conv_fwd(x, weight, bias, ks, stride, pad, keep=keep)
        ctx.save_for_backward(*saved)
        return _as_nchw(y)

    @staticmethod
    def backward(ctx, gy):
        xh, w32 = ctx.saved_tensors
        meta = ctx.meta
        ks, stride, pad, Cin, Cout, H, W, has_bias = meta[:8]
        g = _grad_nhwc(gy, meta)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ks != 7:
                dx = _dx_nchw(_conv_dgrad(g, w32, meta), meta).to(gy.dtype)
            else:  # 7x7 stem input gradient (rarely needed: the input is data)
                dx = torch.nn.grad.conv2d_input((g.shape[0], meta[12], H, W), F.pad(w32, (0, 0, 0, 0, 0,
                                                meta[12] - Cin)).to(gy.dtype), gy[:, :Cout], stride, pad)
        if ctx.needs_input_grad[1]:
            dw = _conv_wgrad(g, xh, meta)
        if has_bias and ctx.needs_input_grad[2]:
            db = gy[:, :Cout].sum((0, 2, 3))
        return dx, dw, db, None, None, None, None


class _NativeConv2dStats(torch.autograd.Function):
    """:class:`_NativeConv2d` that also returns its output's BatchNorm tile statistics (or
    None), computed in the GEMM epilogue: the following training BN skips its statistics pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, ks, stride, pad, keep=False, link_in=None):
        y, saved, ctx.meta, part = _conv_fwd(x, weight, bias, ks, stride, pad, stats=True, keep=keep)
        ctx.save_for_backward(*saved)
        if part is not None:
            ctx.mark_non_differentiable(part)
        # no zero-filled fp64 gradient for the statistics output (one fill launch per conv otherwise)
        ctx.set_materialize_grads(False)
        m = ctx.meta  # a 1x1 stride-1 conv reading its input at its exact width: the producing BN's
        # backward statistics can come from this conv's dgrad epilogue (_BNLink)
        ctx.link_in = link_in if (_BWD_FUSE and ks == 1 and stride == 1 and m[10] == m[12]) else None
        return _as_nchw(y), part

    @staticmethod
    def backward(ctx, gy, _gpart):
        if gy is None:
            return (None,) * 8
        li = ctx.link_in
        if li is None or li.xh is None or not ctx.needs_input_grad[0]:
            return _NativeConv2d.backward(ctx, gy) + (None,)
        xh, w32 = ctx.saved_tensors
        meta = ctx.meta
        if tuple(li.xh.shape) != tuple(xh.shape):
            return _NativeConv2d.backward(ctx, gy) + (None,)
        g = _grad_nhwc(gy, meta)
        dxh, part = _conv_dgrad_fused(g, w32, meta, None, 1, None, li)
        li.part, li.g_ptr, li.g_ver = part, dxh.data_ptr(), dxh._version
        dw = _conv_wgrad(g, xh, meta) if ctx.needs_input_grad[1] else None
        db = gy[:, :meta[4]].sum((0, 2, 3)) if meta[7] and ctx.needs_input_grad[2] else None
        return _dx_nchw(dxh, meta), dw, db, None, None, None, None, None


def _real(x: torch.Tensor, c: int) -> torch.Tensor:
    """The first ``c`` channels of a (possibly padded) activation (the tensor itself if it has c)."""
    return x if x.shape[1] == c else x[:, :c]


def conv_stats(conv: nn.Conv2d, x: torch.Tensor, keep: bool = False, link: _BNLink = None):
    """``(conv(x), tile statistics or None)`` — a native conv whose tuned kernel is a one-pass
    implicit GEMM computes its output's BN statistics in the epilogue (1x1, strided 3x3, the
    packed-tap stem; Winograd picks return None); anything else runs the module (None). ``x`` may
    be a padded activation; ``keep``: the output keeps its carried width (zeros past Cout)."""
    if "forward" in conv.__dict__ and conv.forward.__func__ is _native_forward \
            and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and conv.weight.dtype == torch.float32 \
            and _fits(conv, x):
        ks, s, p = _geom(conv)
        return _NativeConv2dStats.apply(x, conv.weight, conv.bias, ks, s, p, keep, link)
    return conv(_real(x, conv.in_channels)), None


class _NativeBlockEntry(torch.autograd.Function):
    """The two readers of a residual block's input x, as one autograd node: conv1 (1x1, stride 1)
    and the identity branch — x itself, or the downsample conv (1x1, stride s). Returns
    (conv1(x), identity-branch pre-BN). The backward sums the two input gradients inside conv1's
    data-gradient GEMM epilogue (the identity gradient, or the downsample conv's gradient computed
    at its low resolution and scattered to the stride-s pixels), so the separate autograd
    accumulation pass over x (an add kernel per block) disappears."""

    @staticmethod
    def forward(ctx, x, w1, b1, wd, bd, ds_stride, link_in=None, link_res=None):
        # (conv1 output, identity-branch pre-BN, and the two outputs' BN tile statistics or None)
        y1, saved1, ctx.meta1, p1 = _conv_fwd(x, w1, b1, 1, 1, 0, stats=True, keep=True)  # carried width
        ctx.has_ds = wd is not None
        # bottleneck backward fusions (_BNLink): conv1's dgrad output has the block input's exact width
        fuse = _BWD_FUSE and ctx.meta1[10] == ctx.meta1[12] and ctx.meta1[10] % 4 == 0
        ctx.link_in = link_in if fuse else None
        ctx.link_res = link_res if fuse and wd is None else None
        if ctx.link_res is not None:
            link_res.raw_res = True  # read by the block tail's forward (it runs after this node)
        pd = None
        if ctx.has_ds:
            yd, saved_d, ctx.meta_d, pd = _conv_fwd(x, wd, bd, 1, ds_stride, 0, stats=True)
            ctx.save_for_backward(*saved1, saved_d[1])
            out = (_as_nchw(y1), _as_nchw(yd))
        else:
            ctx.save_for_backward(*saved1)
            out = (_as_nchw(y1), x)
        for t in (p1, pd):
            if t is not None:
                ctx.mark_non_differentiable(t)
        ctx.set_materialize_grads(False)  # backward takes None gradients (no fp64 zero fills)
        return out + (p1, pd)

    @staticmethod
    def backward(ctx, g1, gid, _gp1=None, _gpd=None):
        if ctx.has_ds:
            xh, w1, wd = ctx.saved_tensors
        else:
            xh, w1 = ctx.saved_tensors
        m1 = ctx.meta1
        Cx = m1[12]
        dx = dw1 = db1 = dwd = dbd = None
        g1h = _grad_nhwc(g1, m1) if g1 is not None else None
        res, res_stride, gdh, res_bits = None, 1, None, None
        if gid is not None:
            if ctx.has_ds:
                md = ctx.meta_d
                gdh = _grad_nhwc(gid, md)
                if ctx.needs_input_grad[0]:
                    # the strided 1x1 conv's input gradient lives on the stride-s pixels only: the
                    # low-resolution 1x1 GEMM here (stride 1 on the (Ho, Wo) grid), scattered by
                    # conv1's dgrad epilogue
                    res = _conv_dgrad(gdh, wd, (1, 1, 0, md[3], md[4], gdh.shape[1], gdh.shape[2]) + md[7:])
                    res_stride = md[1]
            elif ctx.needs_input_grad[0]:
                res = _nhwc(gid).float()
                if m1[10] != res.shape[-1]:
                    res = F.pad(res, (0, m1[10] - res.shape[-1]))
                res = res.contiguous()
                lr = ctx.link_res
                if lr is not None and lr.raw_res and lr.mk is not None:
                    res_bits, lr.mk = lr.mk, None  # the tail handed its gradient over unmasked
        if ctx.needs_input_grad[0]:
            if g1h is None:  # only the identity branch carries a gradient (rare): dgrad of zeros + res
                B, H, W = xh.shape[0], xh.shape[1], xh.shape[2]
                g1h = torch.zeros((B, H, W, m1[11]), dtype=torch.float32, device=xh.device)
            li = ctx.link_in
            li = li if li is not None and li.xh is not None and tuple(li.xh.shape) == tuple(xh.shape) else None
            if res_bits is not None or li is not None:
                dxh, part = _conv_dgrad_fused(g1h, w1, m1, res, res_stride, res_bits, li)
                if li is not None:
                    li.part, li.g_ptr, li.g_ver = part, dxh.data_ptr(), dxh._version
                dx = _dx_nchw(dxh, m1)
            else:
                dx = _dx_nchw(_conv_dgrad(g1h, w1, m1, res, res_stride), m1)
        if ctx.needs_input_grad[1] and g1 is not None:
            dw1 = _conv_wgrad(g1h, xh, m1)
        if m1[7] and ctx.needs_input_grad[2] and g1 is not None:
            db1 = g1[:, :m1[4]].sum((0, 2, 3))
        if ctx.has_ds and gdh is not None:
            md = ctx.meta_d
            if ctx.needs_input_grad[3]:
                dwd = _conv_wgrad(gdh, xh, md)
            if md[7] and ctx.needs_input_grad[4]:
                dbd = gid.sum((0, 2, 3))
        return dx, dw1, db1, dwd, dbd, None, None, None


class _NativeBN2d(torch.autograd.Function):
    """Training-mode BatchNorm2d on channels_last activations (K5): batch statistics and the
    running-stat update, the normalisation, and the backward, on ``tpamd.bn_train_*``."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, nbt=None, cr=0):
        T = ops.require()
        xh = x.permute(0, 2, 3, 1)
        if not xh.is_contiguous():
            xh = xh.contiguous()
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        y, mean, invstd, _ = T.bn_train_fwd(xh, w, b, running_mean, running_var, float(eps), float(momentum),
                                            num_batches=nbt, cr=int(cr))
        ctx.cr = int(cr)
        if running_mean is not None:
            epochs.bump_stats()  # running stats written by the kernel: no version bump
        ctx.save_for_backward(xh, w if w is not None else torch.empty(0, device=x.device), mean, invstd)
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return _as_nchw(y)

    @staticmethod
    def backward(ctx, gy):
        T = ops.require()
        xh, w, mean, invstd = ctx.saved_tensors
        g = gy.permute(0, 2, 3, 1).contiguous()
        dx, dgamma, dbeta, _ = T.bn_train_bwd(g, xh, w if ctx.has_w else None, mean, invstd,
                                              ctx.needs_input_grad[0], cr=ctx.cr)
        return (dx.permute(0, 3, 1, 2) if ctx.needs_input_grad[0] else None, dgamma if ctx.has_w else None,
                dbeta if ctx.has_b else None, None, None, None, None, None, None)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """(B, H, W, C) contiguous view of a channels_last NCHW tensor (copies otherwise)."""
    th = t.permute(0, 2, 3, 1)
    return th if th.is_contiguous() else th.contiguous()


class _NativeBNAct(torch.autograd.Function):
    """Fused training-mode block tail ``relu?(BN(x) + res?)`` (BN statistics, normalisation,
    residual add and ReLU in one apply pass). The backward masks the gradient by the saved output
    (ReLU), returns it as the residual branch's gradient, and runs the BN backward on it: the
    ATen ReLU / add / threshold-backward passes of the unfused block disappear."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, res, relu, pre=None, nbt=None, cr=0,
                link=None):
        T = ops.require()
        xh = _nhwc(x)
        rh = _nhwc(res) if res is not None else None
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        # cr: the module's channels; x may carry more (a padded activation: zeros, kept zero)
        y, mean, invstd, mk = T.bn_train_fwd(xh, w, b, running_mean, running_var, float(eps), float(momentum), rh,
                                             bool(relu), pre, nbt, int(cr))
        ctx.cr = int(cr)
        ctx.link = None
        if link is not None and relu and xh.shape[-1] % 4 == 0:
            # detached: a link must not reference the graph (a node's ctx holds it: no cycle that would
            # keep old graphs — and their parameters' grad accumulators — alive)
            link.xh, link.mean, link.invstd, link.mk = xh.detach(), mean, invstd, mk
            ctx.link = link
        if running_mean is not None:
            epochs.bump_stats()
        # the backward masks by the ReLU bit mask (1 byte per 4 channels) instead of re-reading y
        ctx.save_for_backward(xh, w if w is not None else torch.empty(0, device=x.device), mean, invstd, mk)
        ctx.has_w, ctx.has_b, ctx.relu, ctx.has_res = weight is not None, bias is not None, relu, res is not None
        return _as_nchw(y)

    @staticmethod
    def backward(ctx, gy):
        T = ops.require()
        xh, w, mean, invstd, mk = ctx.saved_tensors
        g = _nhwc(gy)
        want_res = ctx.has_res and ctx.needs_input_grad[7]
        link, pre = ctx.link, None
        if link is not None and link.part is not None:
            # statistics reduced by the consumer's dgrad epilogue, valid if g is that very output
            # (a second consumer's gradient would have been added in place or into a new tensor)
            if g.data_ptr() == link.g_ptr and g._version == link.g_ver:
                pre = link.part
                FUSE_COUNTS["bn_stats_from_dgrad"] += 1
            link.part = None
        # the entry masks the identity gradient by link.mk (it clears it after use: a second backward
        # over a retained graph runs unfused)
        raw = want_res and link is not None and link.raw_res and link.mk is not None
        if raw:
            FUSE_COUNTS["raw_residual"] += 1
        if link is not None:  # the next block's entry has run: drop the references to this tail's tensors
            link.xh = link.mean = link.invstd = None
        dx, dgamma, dbeta, dres = T.bn_train_bwd(g, xh, w if ctx.has_w else None, mean, invstd,
                                                 ctx.needs_input_grad[0], None, want_res and not raw,
                                                 mk if ctx.relu else None, ctx.cr, pre)
        res_grad = (gy if raw else _as_nchw(dres)) if want_res else None
        return (_as_nchw(dx) if ctx.needs_input_grad[0] else None, dgamma if ctx.has_w else None,
                dbeta if ctx.has_b else None, None, None, None, None, res_grad, None,
                None, None, None, None)


def _bn_counter(bn):
    """The module's ``num_batches_tracked`` when the BN finalize kernel can increment it in place
    (fixed momentum, an int64 GPU scalar): one launch fewer per BN than ``add_(1)``. ``None`` when
    the counter must be bumped on the host side first (cumulative average, momentum=None)."""
    t = bn.num_batches_tracked if bn.track_running_stats else None
    if t is None or bn.momentum is None or not t.is_cuda or t.dtype != torch.int64 or t.numel() != 1:
        return None
    return t


def _bn_fusable(bn, x, res=None) -> bool:
    """Training BN on the native kernels: any width (float4 rows when C % 4 == 0, per-element
    otherwise), x at the module's width or a padded activation carrying more (zeros)."""
    return (isinstance(bn, nn.BatchNorm2d) and bn.training and x.is_cuda and x.dtype == torch.float32
            and x.dim() == 4 and x.shape[1] >= bn.num_features and x.numel() > 0
            and (bn.weight is None or bn.weight.dtype == torch.float32)
            and (res is None or (res.shape == x.shape and res.dtype == x.dtype and res.is_cuda)))


def bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, res: torch.Tensor = None, relu: bool = True,
           pre: torch.Tensor = None, link: _BNLink = None) -> torch.Tensor:
    """``relu?(bn(x) + res?)`` — fused on the native kernels in training mode, the module's own
    ops otherwise (eval mode, unsupported inputs). ``pre``: x's batch statistics already reduced
    per tile by the producing conv's epilogue (:func:`conv_stats`), which skips the statistics
    pass over x. ``link``: a residual block tail's :class:`_BNLink` (bottleneck backward fusions)."""
    if not _bn_fusable(bn, x, res):
        y = bn(_real(x, bn.num_features))
        if res is not None:
            y = y + _real(res, bn.num_features)
        return F.relu(y) if relu else y
    momentum, nbt = bn.momentum, _bn_counter(bn)
    if nbt is None and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        if momentum is None:
            momentum = 1.0 / float(bn.num_batches_tracked)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    if pre is not None and (pre.dim() != 3 or pre.shape[2] != x.shape[1]):
        pre = None
    return _NativeBNAct.apply(x, bn.weight, bn.bias, rm, rv, bn.eps, momentum if momentum is not None else 0.0, res,
                              relu, pre, nbt, bn.num_features, link)


def _block_kind(m) -> str | None:
    """torchvision-layout residual blocks whose training forward can use the fused tails."""
    names = ("conv1", "bn1", "conv2", "bn2", "relu", "downsample")
    if not all(hasattr(m, a) for a in names) or not isinstance(m.relu, nn.ReLU):
        return None
    if hasattr(m, "conv3"):
        return "bottleneck" if isinstance(getattr(m, "bn3", None), nn.BatchNorm2d) else None
    return "basic"


def _entry_convs(block, x):
    """(conv1, downsample conv or None, downsample BN or None) when the block's input readers can
    run as one :class:`_NativeBlockEntry` (1x1 stride-1 conv1; identity or a 1x1 conv + BN
    downsample; fp32 NHWC input), else None."""
    c1, ds = block.conv1, block.downsample
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and isinstance(c1, nn.Conv2d) and eligible(c1)
            and _geom(c1) == (1, 1, 0) and c1.weight.dtype == torch.float32 and _fits(c1, x)):
        return None
    if ds is None:
        return c1, None, None
    if not (type(ds) is nn.Sequential and len(ds) == 2 and isinstance(ds[0], nn.Conv2d) and eligible(ds[0])
            and ds[0].kernel_size == (1, 1) and ds[0].padding == (0, 0) and ds[0].weight.dtype == torch.float32
            and isinstance(ds[1], nn.BatchNorm2d) and _fits(ds[0], x)):
        return None
    return c1, ds[0], ds[1]


def _native_block_forward(self, x):
    """Bottleneck / BasicBlock training forward with fused BN(+residual)+ReLU tails; a
    bottleneck's conv1 and identity branch share one autograd node (:class:`_NativeBlockEntry`),
    whose backward adds the two input gradients inside conv1's dgrad epilogue."""
    if not (self.training and x.is_cuda):
        return type(self).forward(self, x)
    entry = _entry_convs(self, x)
    link = None
    # block-internal activations (conv1 / conv2 outputs: the widths a structured prune cuts) flow at
    # their carried width (_act_w) from conv to BN to conv; the block output has its real width
    if entry is not None:
        c1, dconv, dbn = entry
        # the previous block tail's link (its output is x) and this block's tail link
        link = _BNLink() if _BWD_FUSE and _block_kind(self) == "bottleneck" else None
        y1, idp, p1, pd = _NativeBlockEntry.apply(x, c1.weight, c1.bias, dconv.weight if dconv is not None else None,
                                                  dconv.bias if dconv is not None else None,
                                                  dconv.stride[0] if dconv is not None else 1,
                                                  getattr(x, "_tp_link", None) if _BWD_FUSE else None, link)
        identity = bn_act(dbn, idp, relu=False, pre=pd) if dbn is not None else idp
        out = bn_act(self.bn1, y1, relu=True, pre=p1)
    else:
        identity = self.downsample(x) if self.downsample is not None else x
        y1, p1 = conv_stats(self.conv1, x, keep=True)
        out = bn_act(self.bn1, y1, relu=True, pre=p1)
    if _block_kind(self) == "bottleneck":
        y2, p2 = conv_stats(self.conv2, out, keep=True)
        link2 = _BNLink() if _BWD_FUSE else None  # bn2's backward statistics from conv3's dgrad epilogue
        out = bn_act(self.bn2, y2, relu=True, pre=p2, link=link2)
        y3, p3 = conv_stats(self.conv3, out, link=link2 if link2 is not None and link2.xh is not None else None)
        if link is None and _BWD_FUSE:
            link = _BNLink()  # (no entry node here: the next block can still fuse this tail's statistics)
        out = bn_act(self.bn3, y3, res=identity, relu=True, pre=p3, link=link)
        if link is not None and link.xh is not None:
            out._tp_link = link  # for the next block's entry node (its conv1 dgrad produces our gradient)
        return out
    y2, p2 = conv_stats(self.conv2, out)
    return bn_act(self.bn2, y2, res=identity, relu=True, pre=p2)


# modules a padded activation (zeros past the real width) may pass through unchanged in meaning
_PAD_SAFE = (nn.ReLU, nn.MaxPool2d, nn.Dropout)


def _native_sequential_forward(self, x):
    """nn.Sequential training forward fusing every (BatchNorm2d, ReLU) pair (VGG features). Native
    convs keep their carried output width through BN / ReLU / max-pool / dropout into the next
    conv (no slice / pad copies at pruned widths); any other module gets the real width."""
    mods = list(self.children())
    real = None  # real channel count while x is a padded activation
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.BatchNorm2d) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU) \
                and _bn_fusable(m, x):
            x = bn_act(m, x, relu=True)
            i += 2
            continue
        if "forward" in m.__dict__ and getattr(m.forward, "__func__", None) is _native_forward \
                and self.training and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 \
                and m.weight.dtype == torch.float32 and _fits(m, x):
            ks, s, p = _geom(m)
            x = _NativeConv2d.apply(x, m.weight, m.bias, ks, s, p, True)
            real = m.out_channels if x.shape[1] != m.out_channels else None
            i += 1
            continue
        native_bn = "forward" in m.__dict__ and getattr(m.forward, "__func__", None) is _native_bn_forward
        if real is not None and not (native_bn and _bn_fusable(m, x)) and type(m) not in _PAD_SAFE:
            x, real = x[:, :real], None
        x = m(x)
        i += 1
    return x if real is None else x[:, :real]


def _native_resnet_forward(self, x):
    """ResNet training forward with the stem's BN+ReLU fused (the blocks patch themselves)."""
    if not (self.training and x.is_cuda):
        return type(self).forward(self, x)
    y, p = conv_stats(self.conv1, x)
    x = self.maxpool(bn_act(self.bn1, y, relu=True, pre=p))
    x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
    return self.fc(torch.flatten(self.avgpool(x), 1))


def _native_bn_forward(self, x):
    """BatchNorm2d.forward with the training branch on the native kernels (any width; eval mode and
    inputs the kernels do not take — non-channels_last — use the module's own). A padded activation
    (more channels than the module: zeros) stays padded."""
    ok = (self.training and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
          and x.shape[1] >= self.num_features
          and x.is_contiguous(memory_format=torch.channels_last) and x.numel() > 0
          and (self.weight is None or self.weight.dtype == torch.float32))
    if not ok:
        return type(self).forward(self, x)
    momentum, nbt = self.momentum, _bn_counter(self)
    if nbt is None and self.track_running_stats and self.num_batches_tracked is not None:
        self.num_batches_tracked.add_(1)
        if momentum is None:  # cumulative moving average
            momentum = 1.0 / float(self.num_batches_tracked)
    rm = self.running_mean if self.track_running_stats else None
    rv = self.running_var if self.track_running_stats else None
    return _NativeBN2d.apply(x, self.weight, self.bias, rm, rv, self.eps, momentum if momentum is not None else 0.0,
                             nbt, self.num_features)


class _NativeMaxPool(torch.autograd.Function):
    """Max-pool on NHWC with a window-local argmax byte; backward as a deterministic gather."""

    @staticmethod
    def forward(ctx, x, k, s, pad):
        xh = _nhwc(x)
        y, am = ops.require().maxpool_train_fwd(xh, k, s, pad)
        ctx.save_for_backward(am)
        ctx.geom = (xh.shape[1], xh.shape[2], k, s, pad)
        return _as_nchw(y)

    @staticmethod
    def backward(ctx, gy):
        am, = ctx.saved_tensors
        H, W, k, s, pad = ctx.geom
        return _as_nchw(ops.require().maxpool_train_bwd(_nhwc(gy), am, H, W, k, s, pad)), None, None, None


class _NativeGlobalAvgPool(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) on NHWC: (B, C, 1, 1); backward broadcasts g / HW in one kernel."""

    @staticmethod
    def forward(ctx, x):
        xh = _nhwc(x)
        ctx.hw = (xh.shape[1], xh.shape[2])
        return ops.require().avgpool_nhwc(xh).view(xh.shape[0], xh.shape[3], 1, 1)

    @staticmethod
    def backward(ctx, gy):
        H, W = ctx.hw
        return _as_nchw(ops.require().avgpool_bwd(gy.reshape(gy.shape[0], gy.shape[1]), H, W))


def _pair1(v) -> int | None:
    v = (v, v) if isinstance(v, int) else tuple(v)
    return v[0] if len(v) == 2 and v[0] == v[1] else None


def _cl_f32(x) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] % 4 == 0 and x.numel() > 0
            and x.is_contiguous(memory_format=torch.channels_last))


def _native_maxpool_forward(self, x):
    k, s = _pair1(self.kernel_size), _pair1(self.stride if self.stride is not None else self.kernel_size)
    p, d = _pair1(self.padding), _pair1(self.dilation)
    if not (_cl_f32(x) and k is not None and s is not None and p is not None and d == 1 and not self.ceil_mode
            and not self.return_indices and k * k <= 255 and 2 * p <= k
            and (x.shape[2] + 2 * p - k) // s + 1 > 0 and (x.shape[3] + 2 * p - k) // s + 1 > 0):
        return type(self).forward(self, x)
    return _NativeMaxPool.apply(x, k, s, p)


def _native_gap_forward(self, x):
    if not (_cl_f32(x) and _pair1(self.output_size) == 1):
        return type(self).forward(self, x)
    return _NativeGlobalAvgPool.apply(x)


_MAX_BYTES = (1 << 31) - 1  # the kernels address operands through 32-bit buffer descriptors


def _fits(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    ks, s, p = _geom(conv)
    B, Cin, H, W = x.shape
    Ho, Wo = (H + 2 * p - ks) // s + 1, (W + 2 * p - ks) // s + 1
    cin_p, cout_p = _cin_pad(ks, Cin), _act_w(conv.out_channels)
    return B * H * W * cin_p * 4 <= _MAX_BYTES and B * Ho * Wo * cout_p * 4 <= _MAX_BYTES and Ho > 0 and Wo > 0


class _NativeDropout(torch.autograd.Function):
    """Training-mode inverted dropout on the Philox kernel (K7b): the mask is regenerated from
    (seed, element index) in the backward, nothing is stored."""

    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.p, ctx.seed = p, seed
        return ops.require().dropout(x.contiguous(), seed, p)

    @staticmethod
    def backward(ctx, g):
        return ops.require().dropout(g.contiguous(), ctx.seed, ctx.p), None, None


def _native_dropout_forward(self, x):
    if not (self.training and self.p > 0 and x.is_cuda and x.dtype == torch.float32 and type(self) is nn.Dropout):
        return type(self).forward(self, x)
    if self.p >= 1:
        return x * 0.0
    # seed from torch's CPU generator: reproducible under torch.manual_seed, no device sync
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    y = _NativeDropout.apply(x, float(self.p), seed)
    if self.inplace:
        x.copy_(y)
        return x
    return y


def _native_linear_forward(self, x):
    """nn.Linear on the MFMA GEMM (a 1x1 conv of the (B, 1, 1, in) input): forward, data gradient
    and the weight gradient (pixel-split wgrad kernel) — the classifier of a finetuned model. The
    GEMM shape comes from the weight tensor itself (like F.linear), not from the module's
    ``in_features``/``out_features`` attributes, which user code may leave stale."""
    w = self.weight
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and w.dtype == torch.float32 and w.dim() == 2
            and x.shape[0] > 0 and x.shape[1] == w.shape[1] and (self.bias is None or self.bias.shape == w.shape[:1])
            and x.shape[0] * max(_act_w(w.shape[0]), _act_w(w.shape[1])) * 4 <= _MAX_BYTES):
        return type(self).forward(self, x)
    B, (n_out, n_in) = x.shape[0], w.shape
    y = _NativeConv2d.apply(x.reshape(B, n_in, 1, 1), w.reshape(n_out, n_in, 1, 1), self.bias, 1, 1, 0)
    return y.reshape(B, n_out)


def _native_forward(self, x):
    if not x.is_cuda or x.dtype != torch.float32 or self.weight.dtype != torch.float32 or x.dim() != 4 \
            or not _fits(self, x):
        return type(self).forward(self, x)  # other dtypes / tensors beyond 2 GiB: the library path
    ks, s, p = _geom(self)
    return _NativeConv2d.apply(x, self.weight, self.bias, ks, s, p)


def enable_native_convs(model: nn.Module, bn: bool = True, fuse: bool = True, dropout: bool = True) -> list:
    """Route every eligible ``nn.Conv2d`` of ``model`` (and, with ``bn``, every ``BatchNorm2d`` in
    training mode) through the native kernels (instance-level ``forward`` override; pruning keeps
    working because weights are re-packed per call). With ``bn`` and ``fuse``, residual blocks,
    ResNet stems and ``nn.Sequential`` containers also fuse their BN(+residual)+ReLU tails in
    training mode — the fused BN / ReLU modules (and the convs run by a block's entry node or with
    epilogue BN statistics: a bottleneck's conv1 / downsample, every block's conv2 / conv3, the
    stem conv) are then not called, so forward hooks on them do not fire (attribution passes use
    ``fuse=False``, eval-mode forwards are unchanged). Also switched: ``nn.Linear`` (MFMA GEMM), ``nn.MaxPool2d``,
    ``nn.AdaptiveAvgPool2d`` and, with ``dropout``, training-mode ``nn.Dropout`` (Philox masks
    seeded from torch's CPU RNG: a different random stream than PyTorch's dropout). Returns the
    switched modules; undo with :func:`disable_native_convs`."""
    if not ops.available() or ops.backend() == "torch":
        return []
    from .resnet_engine import _is_resnet
    if not getattr(model, "_tp_pack_epoch_hook", False):  # every forward starts a pack epoch (_PackSet)
        model.register_forward_pre_hook(epochs.bump_fwd)
        model._tp_pack_epoch_hook = True
    switched = []
    for m in model.modules():
        if "forward" in m.__dict__:
            continue
        if bn and fuse and _block_kind(m) is not None:
            m.forward = types.MethodType(_native_block_forward, m)
            switched.append(m)
        elif bn and fuse and _is_resnet(m) and isinstance(m.relu, nn.ReLU) and isinstance(m.bn1, nn.BatchNorm2d):
            m.forward = types.MethodType(_native_resnet_forward, m)
            switched.append(m)
        elif bn and fuse and type(m) is nn.Sequential:
            m.forward = types.MethodType(_native_sequential_forward, m)
            switched.append(m)
        elif eligible(m):
            m.forward = types.MethodType(_native_forward, m)
            switched.append(m)
        elif dropout and type(m) is nn.Dropout:
            m.forward = types.MethodType(_native_dropout_forward, m)
            switched.append(m)
        elif type(m) is nn.Linear:
            m.forward = types.MethodType(_native_linear_forward, m)
            switched.append(m)
        elif type(m) is nn.MaxPool2d:
            m.forward = types.MethodType(_native_maxpool_forward, m)
            switched.append(m)
        elif type(m) is nn.AdaptiveAvgPool2d:
            m.forward = types.MethodType(_native_gap_forward, m)
            switched.append(m)
        elif bn and isinstance(m, nn.BatchNorm2d):
            m.forward = types.MethodType(_native_bn_forward, m)
            switched.append(m)
    return switched


def disable_native_convs(modules) -> None:
    for m in modules:
        m.__dict__.pop("forward", None)


@contextlib.contextmanager
def native_convs(model: nn.Module, enable: bool = True, bn: bool = True, fuse: bool = True, dropout: bool = True):
    """``with native_convs(model): loss.backward()`` — scoped :func:`enable_native_convs`."""
    switched = enable_native_convs(model, bn, fuse, dropout) if enable else []
    try:
        yield switched
    finally:
        disable_native_convs(switched)
