"""Monte-Carlo Shapley values over output units (reference: methods/shapley_values.py:7-99).

Semantics kept from the reference:
* ``sv_samples`` permutations of the ``n`` units are drawn with NumPy's global RNG once
  (on the first batch) and shared by every batch (shapley_values.py:45-47);
* the contribution of unit ``pi[p-1]`` is ``(L_p - L_{p-1}) / S`` where ``L_p`` is the
  per-sample loss with the first ``p`` units of ``pi`` zeroed at the evaluation module;
* fast path via ``model.forward_partial`` when present, slow path (a masking forward hook
  and full forward passes) otherwise.

MI355X-native execution:
* **Batched prefixes.** ``L_p`` for different ``p`` are independent, so K prefixes of one
  permutation are materialised by one HIP launch as a (K*B)-sample batch
  (``ops.prefix_mask``) and evaluated by ONE downstream forward; the K deltas are scattered
  on device (``ops.shapley_scatter`` / ``ops.shapley_column``). The reference runs one tiny
  forward plus one device->host copy per unit (S*n per batch, shapley_values.py:55-61).
  K is sized from an element budget so the batch fills the GPU (288 GB HBM).
* **Work sharding across ranks.** With at least ``world`` batches, whole batches go
  round-robin to ranks and each rank runs its own upstream forward plus every prefix of its
  batches (nothing is replicated); with fewer batches, every rank sees every batch and the
  S*n prefix evaluations are split into contiguous ranges (one boundary evaluation per
  range). Permutations are broadcast from rank 0 (R3); the accumulators are all-reduced
  (stats) or gathered in global batch order (per-sample) once per ``run()`` (R4/R2).
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch
from torch.nn.modules.batchnorm import _BatchNorm
from torch.nn.modules.dropout import _DropoutNd

from ... import ops
from ...parallel import dist as pdist
from ...utils.profiling import trace_range
from ..base import _AttributionMetric

logger = logging.getLogger("torchpruner")


class ShapleyAttributionMetric(_AttributionMetric):
    """Approximate Shapley values by permutation sampling.

    Extra keyword arguments (all optional):
      prefix_batch       fixed number K of prefixes evaluated per forward (default: auto)
      max_eval_elements  element budget used to size K automatically
    """

    def __init__(self, *args, sv_samples=5, prefix_batch=None, max_eval_elements=1 << 29, **kwargs):
        super().__init__(*args, **kwargs)
        self.samples = sv_samples
        self.mask_indices = []
        self.prefix_batch = prefix_batch
        self.max_eval_elements = max_eval_elements

    def run(self, module, sv_samples=None, **kwargs):
        module = super().run(module, **kwargs)
        sv_samples = sv_samples if sv_samples is not None else self.samples
        try:
            return self._run(module, sv_samples)
        finally:
            self._peeked = None  # a batch peeked by the engine selection belongs to this run only

    def _all_batches(self):
        """Every batch with its global index (the prefix-split and single-rank passes)."""
        return ((i, x, y) for i, (x, y) in enumerate(self.data_gen))

    def _peek_source(self):
        return self._source() if self._work_split() == "batches" else self._all_batches()  # hybrid: all

    def _run(self, module, sv_samples):
        why = []
        fused = self._fused_prepare(module, why)
        path = "fused" if fused is not None else None
        if fused is None:
            fused = self._resnet_prepare(module, why)
            path = "resnet" if fused is not None else None
        if fused is not None:
            self._record_path(path, [module], why)
            return self._run_batches(module, sv_samples, fused)
        if hasattr(self.model, "forward_partial"):
            self._record_path("generic-partial", [module], why)
            return self.run_module_with_partial(module, sv_samples)
        self._record_path("generic-hook", [module], why)
        logger.warning("Consider adding a 'forward_partial' method to your model to speed-up Shapley values "
                       "computation")
        return self.run_module(module, sv_samples)

    # ------------------------------------------------------------------ helpers
    def _prefix_chunk(self, B, per_sample):
        if self.prefix_batch is not None:
            return max(1, int(self.prefix_batch))
        if self.model.training and any(isinstance(m, (_BatchNorm, _DropoutNd)) for m in self.model.modules()):
            return 1  # batch statistics / dropout masks would mix across stacked prefixes
        return max(1, int(self.max_eval_elements // max(1, 4 * B * per_sample)))

    def _permutations(self, n, S):
        world, rank = self._world()
        perms = None
        if rank == 0 or world == 1:
            perms = np.stack([np.random.permutation(n) for _ in range(S)]) if S > 0 else np.zeros((0, n), np.int64)
        if world > 1:
            perms = pdist.broadcast_object(perms, 0, self.group)
        return perms

    def _segments(self, S, n, split, K):
        """This rank's share of the flattened (permutation j, prefix p in 1..n) work (all of it
        unless ``split``). The work is cut on the K-prefix chunk grid of the single-rank run
        (chunk c of a permutation covers prefixes c*K+1 .. (c+1)*K), so every stacked
        evaluation has exactly the shape and prefix range it has on one rank and the sharded
        scores are bit-identical to the single-rank ones."""
        world, rank = self._world()
        per = -(-n // K)  # chunks per permutation
        lo, hi = pdist.split_range(S * per, rank, world) if split else (0, S * per)
        segs = []
        c = lo
        while c < hi:
            j, c0 = divmod(c, per)
            c1 = min(per, c0 + (hi - c))  # chunks c0 .. c1-1 of permutation j
            segs.append((j, c0 * K + 1, min(n, c1 * K)))
            c += c1 - c0
        return segs

    def _work_split(self):
        """How ranks share the work: ``"batches"`` — whole batches round-robin, each rank runs
        its own upstream forward and every prefix (scales for deep layers, where the upstream
        forward dominates); ``"prefixes"`` — every rank sees every batch and evaluates a
        contiguous range of the S*n prefixes (when there are fewer batches than ranks);
        ``"hybrid"`` — the first floor(nb/world)*world batches go whole, round-robin, and the
        nb % world remaining ones are prefix-split (10 batches on 8 ranks: 1 whole batch each +
        1/8 of the prefixes of the last 2, instead of 2 ranks with 2 batches and 6 with 1);
        ``None`` — single rank / sharding disabled."""
        world, _ = self._world()
        if world == 1 or self.shard_data is False:
            return None
        if getattr(self.data_gen, "local_only", False):
            # a per-rank loader (ShardLoader) cannot be iterated whole: shard by batches even
            # with fewer batches than ranks (ranks without a batch contribute zeros)
            return "batches"
        try:
            nb = len(self.data_gen)
        except TypeError:
            return "prefixes"
        if nb < world:
            return "prefixes"
        return "batches" if nb % world == 0 else "hybrid"

    @staticmethod
    def _rank_of(perm, device):
        n = len(perm)
        r = torch.empty(n, dtype=torch.int32)
        r[torch.as_tensor(perm, dtype=torch.long)] = torch.arange(n, dtype=torch.int32)
        return r.to(device)

    def _accumulate_permutation(self, perm_t, rank_t, p_lo, p_hi, base_loss, evaluate, K, S, sink):
        """Evaluate prefixes p_lo..p_hi of one permutation and add their deltas to ``sink``.
        Returns the number of prefix image-evaluations made (work accounting)."""
        B = base_loss.shape[0]
        evals = 0
        # a range that starts inside the permutation takes its boundary loss L_{p_lo-1} from the
        # previous full chunk (the same stacked evaluation the single-rank run makes)
        if p_lo == 1:
            prev = base_loss
        else:
            cnt0 = min(K, p_lo - 1)
            prev = evaluate(rank_t, max(1, p_lo - K), cnt0)[-1]
            evals += cnt0 * B
        cur = p_lo
        while cur <= p_hi:
            cnt = min(K, p_hi - cur + 1)
            Ls = evaluate(rank_t, cur, cnt)  # (cnt, B)
            evals += cnt * B
            L = torch.cat([prev.view(1, B), Ls], 0).float().contiguous()
            sink(L, perm_t, cur - 1)
            prev = Ls[-1]
            cur += cnt
        return evals

    def _run_batches(self, module, S, prepare):
        """Shared driver. ``prepare(x, y)`` -> (n, B, per_sample, base_loss, evaluate).

        Batches are "owned" (processed whole by this rank: its share of ``"batches"`` /
        ``"hybrid"``, every batch on one rank) or "replicated" (seen by every rank, each
        evaluating its contiguous share of the prefixes: ``"prefixes"``, the hybrid remainder).
        Owned contributions are summed across ranks with their sample counts; replicated ones
        are partial sums of one result whose count every rank already knows."""
        stats = self.reduction in ("mean", "sum")
        split = self._work_split()
        world, rank = self._world()
        nb_whole = None
        if split == "hybrid":
            nb_whole = (len(self.data_gen) // world) * world
        sv_col = None
        slabs_own, slabs_rep = [], []
        count_own = count_rep = 0
        perms = None
        perm_ts = rank_ts = None
        segs = {}
        work = {"prefix_evals": 0, "upstream_batches": 0}
        if split == "batches":
            batches = self._batches()
        else:
            # hybrid: another rank's whole batch is skipped before its host->device copy
            batches = ((i, _to(x, self.device), _to(y, self.device))
                       for i, x, y in self._iter_source(self._all_batches)
                       if not (split == "hybrid" and i < nb_whole and i % world != rank))
        with torch.no_grad():
            for bidx, x, y in batches:
                replicated = split == "prefixes" or (split == "hybrid" and bidx >= nb_whole)
                if split == "hybrid" and not replicated and bidx % world != rank:
                    continue  # another rank's whole batch
                n, B, per_sample, base_loss, evaluate = prepare(x, y)
                work["upstream_batches"] += 1
                if perms is None:
                    perms = self._permutations(n, S)  # drawn on rank 0, broadcast (R3)
                    perm_ts = [torch.as_tensor(p, dtype=torch.int32).to(base_loss.device) for p in perms]
                    rank_ts = [self._rank_of(p, base_loss.device) for p in perms]
                K = self._prefix_chunk(B, per_sample)
                if (K, replicated) not in segs:
                    segs[(K, replicated)] = self._segments(S, n, replicated, K)
                # deltas are summed unscaled and divided by S at the end. fp64 sums of fp32 loss
                # differences are exact while the exponent span of the terms plus log2(count)
                # stays within fp64's 53 bits, which holds in practice (fp32 losses of one run
                # span far less): then any rank split / collective order gives the same bits
                # (tests/test_loopback_comm.py checks world sizes 1-8)
                if stats:
                    if sv_col is None:
                        sv_col = torch.zeros(n, dtype=torch.float64, device=base_loss.device)
                    sink = lambda L, pt, k0: ops.shapley_column(L, pt, sv_col, k0, 1.0)
                else:
                    slab = torch.zeros(B, n, dtype=torch.float64, device=base_loss.device)
                    (slabs_rep if replicated else slabs_own).append((bidx, slab))
                    sink = lambda L, pt, k0, slab=slab: ops.shapley_scatter(L, pt, slab, 0, k0, 1.0)
                with trace_range("tp.shapley.prefixes"):
                    for j, p_lo, p_hi in segs[(K, replicated)]:
                        work["prefix_evals"] += self._accumulate_permutation(perm_ts[j], rank_ts[j], p_lo, p_hi,
                                                                             base_loss, evaluate, K, S, sink)
                if replicated:
                    count_rep += B
                else:
                    count_own += B
        self.last_work = work
        if split in ("batches", "hybrid") and perms is None:
            self._permutations(0, S)  # a rank without batches still joins the permutation broadcast (R3)
        if stats:
            count = count_own + count_rep
            if split is not None:
                with trace_range("tp.collective"):
                    # ranks agree on n even if one saw no batch; one (n + 1,) fp64 all-reduce (R4)
                    n = pdist.all_max_int(sv_col.numel() if sv_col is not None else 0, self.group)
                    buf = torch.zeros(n + 1, dtype=torch.float64, device=self.device)
                    if sv_col is not None:
                        buf[:n] = sv_col
                    buf[n] = float(count_own)
                    pdist.all_reduce_sum_(buf, self.group)
                    sv_col = buf[:n]
                    count = float(buf[n].item()) + count_rep
            if sv_col is None:
                return np.zeros(0)
            total = sv_col.cpu().numpy() / max(S, 1)
            return total / max(count, 1) if self.reduction == "mean" else total
        parts = []
        if split in ("batches", "hybrid"):
            with trace_range("tp.collective"):
                parts.append(pdist.gather_ordered_rows(slabs_own, self.group))  # global batch order (R2)
        elif slabs_own:
            parts.append(torch.cat([t for _, t in sorted(slabs_own, key=lambda s: s[0])], 0))
        if split in ("prefixes", "hybrid") or slabs_rep:
            rep = torch.cat([t for _, t in slabs_rep], 0) if slabs_rep else torch.zeros(0, 0, dtype=torch.float64)
            if split is not None and rep.numel():
                with trace_range("tp.collective"):
                    pdist.all_reduce_sum_(rep, self.group)
            parts.append(rep)  # the replicated batches are the last ones (hybrid remainder)
        parts = [p for p in parts if p.numel()]
        sv = torch.cat([p.to(parts[0].device) for p in parts], 0) if parts else torch.zeros(0, 0, dtype=torch.float64)
        return self.aggregate_over_samples(sv.cpu().numpy() / max(S, 1))

    # ------------------------------------------------------------------ native path
    def _fused_prepare(self, module, why=None):
        """Prefix evaluation on the fused HIP engine (eval-mode VGG-style chains, any per-sample loss):
        the evaluation module's activation is produced once per batch, K prefix-masked copies
        are stacked by one kernel and pushed through the remaining fused layers in ONE forward.
        Masking a post-ReLU activation commutes with the following 2x2 max-pool, so the
        engine masks its pooled output (4x less data) with identical results."""
        from ...engine.fused_chain import engine_criterion
        fused = self._fused_engine([module], why, need_ce=False, pre_act_ok=True)  # any per-sample criterion
        if fused is None:
            return None
        engine, (k,) = fused
        crit = engine_criterion(self.criterion, self.device)  # None: the fused cross-entropy kernel

        n = engine.real_width(k)
        pad_rank = _RankPadder(n)
        delta = engine.prefix_delta_ok(k)
        perms = {}

        def perm_of(rank_t):  # permutation from its rank vector (cached per rank vector)
            hit = perms.get(id(rank_t))
            if hit is None or hit[0] is not rank_t:
                p = torch.empty_like(rank_t)
                p[rank_t.long()] = torch.arange(rank_t.numel(), dtype=rank_t.dtype, device=rank_t.device)
                hit = perms[id(rank_t)] = (rank_t, p)
            return hit[1]

        def prepare(x, y):
            zk, _ = engine.forward(x, stop_after=k)  # engine layout (B, H, W, C padded)
            B = zk.shape[0]
            z_cl = zk.permute(0, 3, 1, 2)  # (B, C, H, W) view, channels_last strides
            base = engine.loss_from(k, zk, y, crit)
            # masked-copy chunks replay a HIP graph per chunk size (fused cross-entropy only)
            st = engine.shapley_static(k, zk, y) if not delta and crit is None and _graphs_on() else None

            def evaluate(rank_t, p_first, cnt):
                if delta:  # next block is a Linear: prefix-delta GEMM (no masked copies)
                    return engine.prefix_delta_loss(k, zk, perm_of(rank_t), pad_rank(rank_t, zk.shape[3]), p_first,
                                                    cnt, y, crit)
                if st is not None:
                    return engine.shapley_eval(st, pad_rank(rank_t, zk.shape[3]), p_first, cnt)
                masked = ops.prefix_mask(z_cl, pad_rank(rank_t, zk.shape[3]), p_first, cnt)  # channels_last
                loss = engine.loss_from(k, masked.permute(0, 2, 3, 1), y.repeat(cnt), crit)
                return loss.view(cnt, B)

            return n, B, zk[0].numel(), base, evaluate

        return prepare

    def _resnet_prepare(self, module, why=None):
        """Prefix evaluation on the ResNet engine (block-internal BN evaluation modules, any loss):
        the masked activation and the block's residual operand are produced once per batch,
        K prefix-masked copies are pushed through the rest of the block and the network in ONE
        engine forward."""
        from ...engine.fused_chain import engine_criterion, per_sample_loss
        eng = self._resnet_grad_engine([module], why)
        if eng is None:
            return None
        crit = engine_criterion(self.criterion, self.device)  # None: the fused cross-entropy kernel
        bi, ci = eng.locate(module)
        n = module.num_features
        pad_rank = _RankPadder(n)

        def prepare(x, y):
            a, idn = eng.forward_to(x, bi, ci)
            B = a.shape[0]
            a_cl = a.permute(0, 3, 1, 2)
            base = per_sample_loss(eng.logits_from(bi, ci, a, idn), y, crit)

            def evaluate(rank_t, p_first, cnt):
                masked = ops.prefix_mask(a_cl, pad_rank(rank_t, a.shape[3]), p_first, cnt)
                idn_k = idn.repeat(cnt, 1, 1, 1) if cnt > 1 else idn
                loss = per_sample_loss(eng.logits_from(bi, ci, masked.permute(0, 2, 3, 1), idn_k), y.repeat(cnt),
                                       crit)
                return loss.view(cnt, B)

            return n, B, 2 * a[0].numel(), base, evaluate

        return prepare

    # ------------------------------------------------------------------ fast path
    def run_module_with_partial(self, module, sv_samples):
        """Shapley sampling with ``model.forward_partial`` (runs only downstream layers)."""

        def prepare(x, y):
            original_z, _ = self.run_forward_partial(x, to_module=module)
            _, original_loss = self.run_forward_partial(original_z, y_true=y, from_module=module)
            B = original_z.shape[0]
            z = original_z.contiguous() if not original_z.is_contiguous(memory_format=torch.channels_last) \
                else original_z

            def evaluate(rank_t, p_first, cnt):
                masked = ops.prefix_mask(z, rank_t, p_first, cnt)
                yy = y.repeat((cnt,) + (1,) * (y.dim() - 1))
                _, loss = self.run_forward_partial(masked, y_true=yy, from_module=module)
                return loss.reshape(cnt, B, -1).sum(-1)

            return (original_z.shape[1], B, original_z[0].numel(), original_loss.reshape(B, -1).sum(-1), evaluate)

        return self._run_batches(module, sv_samples, prepare)

    # ------------------------------------------------------------------ slow path
    def run_module(self, module, samples):
        """Shapley sampling through full forward passes and a masking forward hook. K prefixes
        are evaluated by ONE forward of the input stacked K times; the hook masks copy k with
        prefix p0 + k (stacking at the module instead would break residual / branching models)."""
        state = {"mode": "off"}

        def hook(_m, _inp, out):
            module._tp_prune_dim = out.shape[1]
            if state["mode"] == "off":
                return None
            return _mask_stacked(out, state["rank"], state["p0"], state["K"])

        handle = module.register_forward_hook(hook)
        try:
            def prepare(x, y):
                self.set_deterministic()
                try:
                    state["mode"] = "off"
                    with self._autocast(), self._native_ctx():
                        out = self.model(x)
                    base = self.criterion(out.float(), y, reduction="none")
                finally:
                    self.restore_deterministic()
                B = x.shape[0]
                n = module._tp_prune_dim

                def evaluate(rank_t, p_first, cnt):
                    state.update(mode="on", rank=rank_t, p0=p_first, K=cnt)
                    self.set_deterministic()
                    try:
                        yy = y.repeat((cnt,) + (1,) * (y.dim() - 1))
                        xx = x.repeat((cnt,) + (1,) * (x.dim() - 1)) if cnt > 1 else x
                        with self._autocast(), self._native_ctx():
                            out = self.model(xx)
                        loss = self.criterion(out.float(), yy, reduction="none")
                    finally:
                        state["mode"] = "off"
                        self.restore_deterministic()
                    return loss.reshape(cnt, B, -1).sum(-1)

                return n, B, max(1, x[0].numel()), base.reshape(B, -1).sum(-1), evaluate

            return self._run_batches(module, samples, prepare)
        finally:
            handle.remove()
            if hasattr(module, "_tp_prune_dim"):
                delattr(module, "_tp_prune_dim")
            self.mask_indices = []

    def _forward_hook(self):
        """Reference-compatible masking hook: zero ``self.mask_indices`` of the output."""
        def _hook(module, _, output):
            module._tp_prune_dim = output.shape[1]
            return output.index_fill_(1, torch.tensor(self.mask_indices, dtype=torch.long,
                                                      device=output.device), 0.0)
        return _hook


def _mask_stacked(out, rank, p0, K):
    """``out`` holds K stacked copies (K*B, C, ...): zero, in copy k, the channels of rank <
    p0 + k (exact zeros, as index_fill_ in the reference)."""
    C = out.shape[1]
    ks = torch.arange(K, device=out.device).view(K, 1) + p0
    keep = rank.to(out.device).view(1, C) >= ks  # (K, C)
    o = out.reshape((K, -1) + tuple(out.shape[1:]))
    keep = keep.view((K, 1, C) + (1,) * (out.dim() - 2))
    return torch.where(keep, o, torch.zeros((), dtype=out.dtype, device=out.device)).reshape(out.shape)


def _graphs_on() -> bool:
    """HIP-graph replay of the fused engine's prefix chunks (TORCHPRUNER_GRAPHS != "0")."""
    return os.environ.get("TORCHPRUNER_GRAPHS", "auto") != "0"


class _RankPadder:
    """Rank vectors over ``n`` real units extended to the engine's channel-padded width: padding
    channels rank after every real unit, so no prefix ever masks them (cached per rank vector)."""

    def __init__(self, n):
        self.n = n
        self.cache = {}

    def __call__(self, rank_t, width):
        pad = width - self.n
        if pad <= 0:
            return rank_t
        r = self.cache.get(id(rank_t))
        if r is None or r[0] is not rank_t:
            r = self.cache[id(rank_t)] = (rank_t, torch.cat([rank_t, torch.full(
                (pad,), self.n + 1, dtype=rank_t.dtype, device=rank_t.device)]))
        return r[1]


def _to(t, device):
    return t.to(device, non_blocking=True) if isinstance(t, torch.Tensor) else t
