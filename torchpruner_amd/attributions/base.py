"""Attribution-metric core (reference: torchpruner/attributions/attributions.py:15-116).

Same public contract as the reference — ``Metric(model, data_generator, criterion, device,
reduction="mean", ...)`` and ``run(module, find_best_evaluation_module=False)`` returning a
NumPy array — re-designed for MI355X:

* **Device-resident accumulation.** Hooks never copy to the host. Per-sample (B, C) scores
  are produced by the HIP channel-reduction kernels (ops.channel_reduce) and folded into
  float64 device accumulators (ops.column_accumulate); one device->host copy per ``run()``.
  The reference does ``.cpu().numpy()`` + ``np.concatenate`` on every batch (O(N^2) host
  work, a device sync per batch — apoz.py:34-38, taylor.py:46-48).
* **Data parallel.** When a process group is live, whole batches are sharded round-robin
  over ranks (parallel.dist.ShardedBatches) and the (C+1,) accumulator is all-reduced once
  per ``run()`` over RCCL (R1); per-sample slabs for ``reduction="none"``/callables are
  all-gathered in global batch order (R2).
* **Gradient capture by tensor hooks** on a fresh leaf that replaces the evaluation module's
  output (safe with ``ReLU(inplace=True)``, which the deprecated non-full
  ``register_backward_hook`` of the reference relies on). Parameters are frozen during the
  pass, so backward runs only downstream of the evaluation module and only the input
  gradients (no weight-gradient GEMMs). Scores are identical to the reference; the
  reference's side effect of accumulating ``param.grad`` is intentionally dropped.
"""
from __future__ import annotations

import contextlib
import itertools
import logging
import math
import os
from abc import ABC, abstractmethod

import numpy as np
import torch
import torch.nn as nn
from torch.nn.modules.conv import _ConvNd

from .. import ops
from ..data.prefetch import prefetch_to_device
from ..parallel import dist as pdist
from ..utils.graph import ACTIVATIONS, find_best_module_for_attributions
from ..utils.profiling import range_pop, range_push, trace_range

logger = logging.getLogger("torchpruner")

SUPPORTED_OUT_PRUNING_MODULES = [nn.Linear, _ConvNd]
__all__ = ["_AttributionMetric", "SUPPORTED_OUT_PRUNING_MODULES", "ACTIVATIONS", "ScoreAccumulator"]


class ScoreAccumulator:
    """Per-unit score accumulator living on the metric's device.

    ``stats`` mode (reduction mean/sum): float64 (C,) running sum + sample count.
    ``samples`` mode (reduction none/callable): the per-batch (B, C) slabs, kept on device
    and tagged with their global batch index so data-parallel gathers preserve order.
    """

    def __init__(self, reduction, device):
        self.mode = "stats" if reduction in ("mean", "sum") else "samples"
        self.device = torch.device(device)
        self.sum = None
        self.count = 0
        self.slabs: list[tuple[int, torch.Tensor]] = []
        self.dtype = None
        self.width = None  # real unit count when the engine's slabs are channel-padded

    def ensure_sum(self, C: int, device, width=None) -> torch.Tensor:
        """The fp64 (C,) running sum (allocated on first use) for kernels that fold into it;
        ``width`` < C marks the trailing C - width entries as engine padding (dropped on output)."""
        if self.sum is None:
            self.sum = torch.zeros(C, dtype=torch.float64, device=device)
            self.dtype = torch.float32
            self.width = width
        return self.sum

    def add(self, v: torch.Tensor, batch_index: int):
        """Add a (B, C) per-sample score slab for global batch ``batch_index``."""
        if self.dtype is None:
            self.dtype = v.dtype
        if self.mode == "stats":
            if self.sum is None:
                self.sum = torch.zeros(v.shape[1], dtype=torch.float64, device=v.device)
            ops.column_accumulate(v, self.sum)
            self.count += v.shape[0]
        else:
            self.slabs.append((batch_index, v.detach()))

    def finalize(self, reduction, aggregate, collective=False, group=None):
        """Reduce across ranks (if ``collective``) and apply ``reduction``; returns NumPy."""
        if not collective:
            return self._finalize_local(reduction, aggregate)
        with trace_range("tp.collective"):
            return self._finalize_collective(reduction, aggregate, group)

    def _finalize_collective(self, reduction, aggregate, group):
        out_dtype = np.float32 if self.dtype in (None, torch.float32, torch.float16, torch.bfloat16) else np.float64
        if self.mode == "stats":
            n = self.sum.numel() if self.sum is not None else 0
            # ranks must agree on C even if one owned no batches: share it first
            n = pdist.all_max_int(n, group)
            buf = torch.zeros(n + 1, dtype=torch.float64, device=self.device)
            if self.sum is not None:
                buf[:n] = self.sum
            buf[n] = float(self.count)
            pdist.all_reduce_sum_(buf, group)
            host = buf.cpu().numpy()
            total, count = host[:n], host[n]
            if reduction == "mean":
                res = total / max(count, 1.0)
            else:
                res = total
            return res[:self.width].astype(out_dtype)
        rows = pdist.gather_ordered_rows(self.slabs, group)
        return self._to_numpy_rows(rows, aggregate, out_dtype)

    def _finalize_local(self, reduction, aggregate):
        out_dtype = np.float32 if self.dtype in (None, torch.float32, torch.float16, torch.bfloat16) else np.float64
        if self.mode == "stats":
            total = self.sum.cpu().numpy() if self.sum is not None else np.zeros(0)
            res = total / max(self.count, 1) if reduction == "mean" else total
            return res[:self.width].astype(out_dtype)
        slabs = sorted(self.slabs, key=lambda s: s[0])
        rows = torch.cat([t for _, t in slabs], 0) if slabs else torch.empty(0)
        return self._to_numpy_rows(rows, aggregate, out_dtype)

    @staticmethod
    def _to_numpy_rows(rows, aggregate, out_dtype):
        arr = rows.cpu().numpy()
        if arr.dtype != out_dtype and out_dtype == np.float32:
            arr = arr.astype(np.float32)
        return aggregate(arr)


class _AttributionMetric(ABC):
    """Abstract base of every metric (reference attributions.py:15-25)."""

    def __init__(self, model, data_generator, criterion, device, reduction="mean", *, group=None,
                 shard_data=None, checkpoint=None, checkpoint_every=50, compute_dtype=None):
        assert reduction in ["mean", "none", "sum"] or callable(reduction), \
            'Reduction must be a string in ["mean", "none", "sum"] or a function'
        self.model = model
        self.data_gen = data_generator
        self.criterion = criterion
        self.device = device
        self.reduction = reduction
        self.deterministic = False
        self.benchmark = False
        # Data-parallel knobs (new): process group and whether to shard the generator.
        # shard_data=None -> shard automatically when a multi-rank group is live.
        self.group = group
        self.shard_data = shard_data
        # Resume support (new): accumulators + processed batch indices are persisted every
        # ``checkpoint_every`` batches to ``checkpoint`` (a per-rank path in DP runs).
        self.checkpoint = checkpoint
        self.checkpoint_every = checkpoint_every
        # dtype policy (new): None / float32 = exact fp32 (the reference's precision; the fused
        # engines apply); bfloat16 / float16 = opt-in autocast of the model's forward passes on
        # the generic path (scores are still reduced and accumulated in fp32/fp64)
        assert compute_dtype in (None, torch.float32, torch.bfloat16, torch.float16), \
            "compute_dtype must be None, torch.float32, torch.bfloat16 or torch.float16"
        self.compute_dtype = compute_dtype
        self._ckpt = None
        self._run_accs = None
        self._peeked = None  # (first batch, live iterator) taken by _first_input_shape
        # path transparency (new): which execution path served the last run() and, when the
        # generic hook path ran, why the native engines were rejected
        self.last_path = None

    # ------------------------------------------------------------------ API parity
    @abstractmethod
    def run(self, module, **kwargs):
        assert any(isinstance(module, t) for t in SUPPORTED_OUT_PRUNING_MODULES), \
            f"Attributions can be computed only for the following modules {SUPPORTED_OUT_PRUNING_MODULES}"
        return self.find_evaluation_module(module, **kwargs)

    def find_evaluation_module(self, module, find_best_evaluation_module=False):
        if find_best_evaluation_module is True:
            return find_best_module_for_attributions(self.model, module)
        return module

    def run_all_forward(self):
        """No-grad forward over this rank's batches; returns per-sample losses (concatenated)."""
        self.set_deterministic()
        losses = []
        try:
            with torch.no_grad(), self._native_ctx():
                for _, x, y in self._batches():
                    with self._autocast():
                        out = self.model(x)
                    losses.append(self.criterion(out.float(), y, reduction="none"))
        finally:
            self.restore_deterministic()
        return torch.cat(losses, 0) if losses else None

    def run_all_forward_and_backward(self):
        """Forward + backward (default mean reduction) over this rank's batches."""
        self.set_deterministic()
        try:
            for _, x, y in self._batches():
                with self._autocast(), self._native_ctx():
                    out = self.model(x)
                    loss = self.criterion(out.float(), y)
                    loss.backward()
        finally:
            self.restore_deterministic()

    def run_forward_partial(self, x=None, y_true=None, to_module=None, from_module=None):
        """``model.forward_partial`` wrapper (attributions.py:70-89)."""
        self.set_deterministic()
        loss = None
        try:
            with self._autocast(), self._native_ctx():
                y = self.model.forward_partial(x, to_module=to_module, from_module=from_module)
            if y_true is not None and to_module is None:
                loss = self.criterion(y.float(), y_true, reduction="none")
        finally:
            self.restore_deterministic()
        return y, loss

    def aggregate_over_samples(self, attributions):
        """Host NumPy aggregation over axis 0 (attributions.py:91-106)."""
        if self.reduction == "mean":
            return np.mean(attributions, 0)
        elif self.reduction == "sum":
            return np.sum(attributions, 0)
        elif self.reduction == "none":
            return attributions
        return self.reduction(attributions)

    def set_deterministic(self):
        """Reference parity (attributions.py:108-112) with one ROCm-specific deviation.

        On ROCm ``cudnn.deterministic=True`` selects MIOpen's deterministic solvers, which are
        ~76x slower for ResNet-50 forward (measured on MI355X) and buy nothing here: attribution
        passes compute no weight gradients (the only atomic-reduction convolutions), MIOpen's
        immediate-mode forward/data-gradient solvers are already run-to-run deterministic, and
        the fused HIP engine is deterministic by construction. The flag is therefore only forced
        on ROCm when ``TORCHPRUNER_DETERMINISTIC=1``; it is always saved and restored.
        """
        self.deterministic = torch.backends.cudnn.deterministic
        self.benchmark = torch.backends.cudnn.benchmark
        if torch.version.hip is None or os.environ.get("TORCHPRUNER_DETERMINISTIC", "0") == "1":
            torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False

    def restore_deterministic(self):
        torch.backends.cudnn.deterministic = self.deterministic
        torch.backends.cudnn.benchmark = self.benchmark

    # ------------------------------------------------------------------ engine internals
    def _native_ctx(self):
        """Generic path on the native kernels: every eligible ``nn.Conv2d``, ``nn.Linear``,
        ``nn.MaxPool2d``, ``nn.AdaptiveAvgPool2d`` and training-mode ``BatchNorm2d`` of the model
        runs the HIP kernels through autograd instead of MIOpen / hipBLASLt, unfused so that every
        module's hooks fire (TORCHPRUNER_GENERIC_NATIVE=0 disables; reduced compute dtypes keep
        autocast). ``nn.Dropout`` stays on PyTorch: a model scored in training mode draws its
        dropout masks from the same RNG stream as with the reference."""
        from ..engine.train import native_convs
        enable = (torch.device(self.device).type == "cuda" and not self._reduced_precision()
                  and os.environ.get("TORCHPRUNER_GENERIC_NATIVE", "1") != "0" and ops.backend() != "torch")
        return native_convs(self.model, enable=enable, fuse=False, dropout=False)  # hooks must see every module

    def _record_path(self, path: str, eval_modules, why=()):
        """Remember and log (once per run, ``torchpruner`` logger) which path served it:
        ``fused`` (VGG-chain engine), ``resnet`` (ResNet engine) or ``generic`` (PyTorch
        modules + HIP reduction kernels), with the engines' rejection reasons."""
        names = {id(m): n for n, m in self.model.named_modules()}
        mods = [names.get(id(m), type(m).__name__) for m in eval_modules]
        reasons = [r for r in dict.fromkeys(why or ())]
        self.last_path = {"path": path, "modules": mods, "reasons": reasons}
        if path.startswith("generic") and torch.device(self.device).type == "cuda":
            from ..engine.train import eligible
            self.last_path["native_convs"] = sum(eligible(m) for m in self.model.modules()) \
                if os.environ.get("TORCHPRUNER_GENERIC_NATIVE", "1") != "0" and not self._reduced_precision() else 0
        msg = f"{type(self).__name__}: {path} path for {', '.join(mods)}"
        if reasons:
            msg += " (" + "; ".join(reasons) + ")"
        logger.info(msg)

    def _reduced_precision(self) -> bool:
        return self.compute_dtype in (torch.bfloat16, torch.float16)

    def _engines_allowed(self) -> bool:
        """The fused HIP engines compute in exact fp32; a reduced compute dtype uses the
        generic (autocast) path instead."""
        return not self._reduced_precision()

    def _autocast(self):
        if not self._reduced_precision():
            return contextlib.nullcontext()
        return torch.autocast(device_type=torch.device(self.device).type, dtype=self.compute_dtype)

    def _world(self):
        return pdist.get_world_size(self.group), pdist.get_rank(self.group)

    def _sharding(self) -> bool:
        world, _ = self._world()
        return world > 1 and (self.shard_data is None or self.shard_data)

    def _source(self):
        """This rank's ``(global_batch_index, x, y)`` batches, straight from the data generator."""
        world, rank = self._world()
        return pdist.ShardedBatches(self.data_gen, rank, world) if self._sharding() else \
            ((i, x, y) for i, (x, y) in enumerate(self.data_gen))

    def _peek_source(self):
        """The batch iterator the coming pass will consume (``_first_input_shape`` peeks it)."""
        return self._source()

    def _iter_source(self, factory):
        """The peeked iterator (its first batch replayed) if the engine selection took one, else
        ``factory()``: the data generator is iterated once per pass."""
        peeked, self._peeked = getattr(self, "_peeked", None), None
        if peeked is not None:
            return itertools.chain([peeked[0]], peeked[1])
        return factory()

    def _batches(self):
        """Yield ``(global_batch_index, x, y)`` on ``self.device`` for this rank's batches. A
        batch the engine selection peeked at (``_first_input_shape``) is replayed first, from the
        same iterator: the data generator is iterated once per pass, as by the reference."""
        it = self._iter_source(self._source)
        ck = self._ckpt
        if ck is not None:
            it = ((i, x, y) for i, x, y in it if i not in ck.done)  # processed before an interruption
        # host batches are pinned and copied one batch ahead on a side stream (copy/compute overlap)
        for i, x, y in prefetch_to_device(it, self.device):
            yield i, x, y
            if ck is not None:  # the consumer finished batch i before asking for the next one
                ck.step(self._run_accs, i)

    def _new_accumulator(self) -> ScoreAccumulator:
        return ScoreAccumulator(self.reduction, self.device)

    def _begin_run(self, accs, eval_modules):
        """Attach (and restore) the resumable checkpoint of this run, if configured."""
        self._run_accs = accs
        self._ckpt = None
        self._range = range_push(f"tp.run/{type(self).__name__}")
        if self.checkpoint:
            from ..checkpoint import AttributionCheckpoint
            names = {id(m): n for n, m in self.model.named_modules()}
            key = "|".join([type(self).__name__, str(self.reduction), str(getattr(self, "signed", ""))] +
                           [names.get(id(m), type(m).__name__) for m in eval_modules])
            world, rank = self._world()
            path = self.checkpoint if world == 1 else f"{self.checkpoint}.rank{rank}"
            self._ckpt = AttributionCheckpoint(path, key, self.checkpoint_every)
            self._ckpt.restore(accs)

    def _end_run(self):
        self._peeked = None  # a peeked batch belongs to this run's pass only
        if self._ckpt is not None:
            self._ckpt.save(self._run_accs)
        self._ckpt = None
        self._run_accs = None
        range_pop(getattr(self, "_range", False))
        self._range = False

    def _finalize(self, acc: ScoreAccumulator):
        # not sharded: every rank already holds the full result, so no collective
        return acc.finalize(self.reduction, self.aggregate_over_samples, collective=self._sharding(),
                            group=self.group)

    @contextlib.contextmanager
    def _frozen_params(self):
        """Temporarily stop every parameter from requiring grad (input-grad-only backward)."""
        flags = [(p, p.requires_grad) for p in self.model.parameters()]
        for p, _ in flags:
            p.requires_grad_(False)
        try:
            yield
        finally:
            for p, f in flags:
                p.requires_grad_(f)

    def _has_inplace(self) -> bool:
        return any(getattr(m, "inplace", False) for m in self.model.modules())

    def _grad_capture_pass(self, eval_modules, on_grad):
        """Forward+backward over this rank's batches capturing, for every module in
        ``eval_modules``, its output ``a`` and ``dL/da``: ``on_grad(k, a, g, batch_index)``.

        The first evaluation module to execute becomes the autograd leaf (nothing upstream
        is differentiated); parameters are frozen so only input gradients are computed.
        One pass serves any number of modules (the reference needs one pass per module).
        """
        if isinstance(eval_modules, nn.Module):
            eval_modules = [eval_modules]
        state = {}
        has_inplace = self._has_inplace()

        def make_hook(k, module):
            # an activation's consumers are convs/pools/linears; a conv/linear/BN output may be
            # consumed by an in-place activation, so hand a copy downstream in that case
            copy_out = has_inplace and not isinstance(module, ACTIVATIONS)

            def fwd_hook(_m, _inp, out):
                idx = state["idx"]
                if not state["leafed"]:
                    state["leafed"] = True
                    src = out.detach().requires_grad_(True)
                    ret = src.clone() if (copy_out or has_inplace) else src
                else:
                    src = out
                    ret = out.clone() if copy_out else None
                act = src.detach()
                version = act._version

                def _tensor_hook(g):
                    if act._version != version:
                        raise RuntimeError(
                            f"activation of {module} was modified in place after capture; "
                            "attribute at a different module")
                    on_grad(k, act, g, idx)
                src.register_hook(_tensor_hook)
                return ret

            return fwd_hook

        handles = [m.register_forward_hook(make_hook(k, m)) for k, m in enumerate(eval_modules)]
        self.set_deterministic()
        try:
            with self._frozen_params(), self._native_ctx():
                for i, x, y in self._batches():
                    state["idx"] = i
                    state["leafed"] = False
                    with self._autocast():
                        out = self.model(x)
                    loss = self.criterion(out.float(), y)
                    loss.backward()
        finally:
            for h in handles:
                h.remove()
            self.restore_deterministic()

    # Small loader batches on the fused engine are coalesced: ~COALESCE_ELEMS input elements per
    # engine launch (B=100 at 3x32x32 -> 5 loader batches = 500 images per launch). In eval mode every
    # sample's forward / backward is independent of the others in its batch and the fused
    # cross-entropy keeps each loader batch's 1/B loss scaling, so every per-sample score is the one
    # its own batch gives (up to kernel-choice rounding); scores are folded per sample, |.| included.
    # TORCHPRUNER_COALESCE=0 turns it off; =k (k >= 2) coalesces k loader batches per launch.
    COALESCE_ELEMS = 3 << 19

    def _coalesce_factor(self, x) -> int:
        env = os.environ.get("TORCHPRUNER_COALESCE", "1")
        if env == "0" or not x.is_cuda:
            return 1
        if env.isdigit() and int(env) >= 2:
            return int(env)
        return max(1, self.COALESCE_ELEMS // max(1, x.shape[0] * math.prod(x.shape[1:])))

    def _coalesced_batches(self, on: bool, max_batch=None):
        """``(global_batch_index, x, y, loss_batch)`` over this rank's batches; with ``on``, runs of
        k equal-shape batches come concatenated (``loss_batch`` = the loader batch size, the
        group's first index), leftovers and odd shapes alone (``loss_batch`` None).
        ``max_batch(x) -> int``: a batch larger than that is run in slices (every slice with the
        whole batch's loss scaling): the kernels' buffer descriptors address < 2^31 bytes."""
        self.last_coalesce = 1
        for i, x, y, lb in self._coalesced_groups(on):
            mb = max_batch(x) if max_batch is not None else x.shape[0]
            if x.shape[0] <= mb:
                yield i, x, y, lb
                continue
            n = -(-x.shape[0] // mb)
            step = -(-x.shape[0] // n)  # equal slices (one shape to tune, no 1-image tail)
            for s in range(0, x.shape[0], step):
                yield i, x[s:s + step], y[s:s + step], lb or x.shape[0]

    def _coalesced_groups(self, on: bool):
        if not on:
            for i, x, y in self._batches():
                yield i, x, y, None
            return
        group, k = [], 1
        for i, x, y in self._batches():
            if group and (x.shape != group[0][1].shape or y.shape != group[0][2].shape):
                for g in group:  # a batch of another shape (the last one): no partial groups
                    yield g + (None,)
                group = []
            if not group:
                k = self._coalesce_factor(x)
            group.append((i, x, y))
            if len(group) < k:
                continue
            if k == 1:
                yield i, x, y, None
            else:
                self.last_coalesce = k
                yield group[0][0], torch.cat([g[1] for g in group]), torch.cat([g[2] for g in group]), x.shape[0]
            group = []
        for g in group:
            yield g + (None,)

    def _fused_grad_pass(self, engine, blocks, accs, mode, take_abs):
        """Gradient metrics on the fused VGG-chain engine: per batch ONE fused forward +
        input-gradient backward writes every block's per-sample partials (``mode`` taylor /
        sensitivity), and ONE fold launch turns all layers' sums into fp64 accumulators. Small
        batches are coalesced (see COALESCE_ELEMS) and pipelined over HIP streams."""
        from ..engine.fused_chain import engine_criterion
        owner = {}
        for k, b in enumerate(blocks):
            owner.setdefault(b, k)
        uniq = sorted(owner)
        stats = accs[0].mode == "stats"
        crit = engine_criterion(self.criterion, self.device)  # None: the fused cross-entropy kernel
        pipe = _BatchPipeline(engine, graph_replay=True) if stats and self._ckpt is None and crit is None else None

        def run_batch(i, x, y, loss_batch=None):
            B = x.shape[0]

            def launch(slot, x=x, y=y):
                arena = engine.score_arena(x.shape[0], uniq, x.device, tuple(x.shape[2:]), slot=slot)
                if engine.graphs_enabled(x.shape[0], pipelined=True):  # host-bound otherwise
                    engine.taylor_graphed(x, y, set(uniq), arena, mode=mode, warm=True, loss_batch=loss_batch)
                else:
                    engine.taylor(x, y, set(uniq), arena, mode=mode, loss_batch=loss_batch)
                return arena

            def fold(arena, dev=x.device):
                sums = [accs[owner[b]].ensure_sum(arena[b].shape[-1], dev, engine.real_width(b)) for b in uniq]
                ops.score_fold_([arena[b] for b in uniq], sums, take_abs, 2)

            if pipe is not None and pipe.take(x, y, launch, fold):
                for b in uniq:
                    accs[owner[b]].count += B
                return
            if stats:
                arena = engine.score_arena(B, uniq, x.device, tuple(x.shape[2:]))
                with trace_range("tp.forward_backward"):
                    if engine.graphs_enabled(B):  # small batches are launch-bound: replay a HIP graph
                        engine.taylor_graphed(x, y, set(uniq), arena, mode=mode, criterion=crit, loss_batch=loss_batch)
                    else:
                        engine.taylor(x, y, set(uniq), arena, mode=mode, criterion=crit, loss_batch=loss_batch)
                sums = [accs[owner[b]].ensure_sum(arena[b].shape[-1], x.device, engine.real_width(b)) for b in uniq]
                with trace_range("tp.fold"):
                    ops.score_fold_([arena[b] for b in uniq], sums, take_abs, 2)
                for b in uniq:
                    accs[owner[b]].count += B
            else:
                res = engine.taylor(x, y, set(uniq), mode=mode, criterion=crit, loss_batch=loss_batch)
                ops.score_fold_([res[b] for b in uniq], [None] * len(uniq), take_abs, 1)
                for b in uniq:
                    accs[owner[b]].add(engine.per_sample(res[b])[:, :engine.real_width(b)], i)

        big = (lambda x: engine.max_batch(tuple(x.shape[1:]))) if crit is None else None
        try:
            for i, x, y, lb in self._coalesced_batches(pipe is not None, big):
                run_batch(i, x, y, lb)
        finally:  # the tuner's in-flight concurrency is reset even if a batch raises
            if pipe is not None:
                pipe.join()
        return [accs[owner[b]] for b in blocks]

    def _resnet_grad_engine(self, eval_modules, why=None):
        """The ResNet engine when it can produce gradient scores for ``eval_modules`` (eval-mode
        torchvision-layout ResNet, block BNs; any differentiable criterion), else None."""
        from ..engine.fused_chain import _reject
        from ..engine.resnet_engine import maybe_resnet_engine
        if not self._engines_allowed():
            return _reject(why, f"compute_dtype={self.compute_dtype} runs the generic autocast path")
        return maybe_resnet_engine(self.model, eval_modules, self.device, grad=True, why=why)

    def _fused_engine(self, eval_modules, why=None, need_ce=True, pre_act_ok=False):
        """The fused chain engine (engine, block indices) for ``eval_modules``, else None.
        ``compute_dtype=torch.bfloat16`` runs it with bf16-operand 3x3 convs (fp32 accumulation,
        fp32 activations / gradients, fp64 score accumulators); fp16 uses the generic path."""
        from ..engine.fused_chain import _reject, maybe_engine
        bf16 = self.compute_dtype == torch.bfloat16
        if not self._engines_allowed() and not bf16:
            return _reject(why, f"compute_dtype={self.compute_dtype} runs the generic autocast path")
        res = maybe_engine(self.model, eval_modules, self.criterion, self.device, need_ce=need_ce, why=why,
                           pre_act_ok=pre_act_ok, input_shape=self._agreed_input_shape())
        if res is not None:
            res[0].bf16 = bf16
        return res

    def _agreed_input_shape(self):
        """``_first_input_shape`` made rank-consistent under data-parallel sharding: a rank whose
        shard is empty (fewer batches than ranks) peeks nothing, so every rank takes the first
        non-empty rank's shape (one all_gather_object) and all ranks make the same fused / generic
        decision (``last_path`` could otherwise differ across ranks)."""
        shape = self._first_input_shape()
        world, _ = self._world()
        if world > 1 and self._sharding():
            shapes = pdist.all_gather_object(shape, group=self.group)
            shape = next((tuple(s_) for s_ in shapes if s_ is not None), None)
        return shape

    def _first_input_shape(self):
        """Shape of this rank's first input batch, or None. In-memory loaders (DeviceLoader,
        per-rank ShardLoader) are indexed without iterating. Anything else is iterated ONCE, here:
        the first batch and the live iterator are kept for the pass that follows (``_batches``),
        so a DataLoader is not iterated twice (a second iterator would draw its shuffle seed and
        start its workers again, shifting the RNG stream the reference's single pass sees) and a
        one-shot iterable loses nothing."""
        peeked = getattr(self, "_peeked", None)
        if peeked is None:
            dg = self.data_gen
            x = None
            if getattr(dg, "local_only", False):  # a per-rank ShardLoader
                first = next(iter(dg.batches.values()), None)
                x = first[0] if first else None
            elif hasattr(dg, "_batch") and hasattr(dg, "x"):  # DeviceLoader: resident tensors
                x = dg._batch(0)[0] if len(dg) else None
            else:
                it = iter(self._peek_source())
                first = next(it, None)
                if first is None:
                    return None
                self._peeked = peeked = (first, it)
            if peeked is None:
                return tuple(x.shape) if isinstance(x, torch.Tensor) else None
        x = peeked[0][1]
        return tuple(x.shape) if isinstance(x, torch.Tensor) else None

    def _resnet_grad_pass(self, eng, eval_modules, accs, mode):
        """Per batch: one engine forward + input-gradient backward scores every module; the
        (B, C_padded) slabs are folded into fp64 accumulators (16 layers per launch)."""
        from ..engine.fused_chain import engine_criterion
        uniq = list(dict.fromkeys(eval_modules))
        first = {}
        for k, m in enumerate(eval_modules):
            first.setdefault(m, k)
        stats = accs[0].mode == "stats"
        crit = engine_criterion(self.criterion, self.device)  # None: the fused cross-entropy kernel
        pipe = _BatchPipeline(eng) if stats and self._ckpt is None and crit is None else None
        # batches past the kernels' descriptor range run in slices (whole-batch loss scaling)
        big = (lambda x: eng.max_batch(tuple(x.shape[1:]))) if crit is None else None
        try:
            with torch.no_grad():
                # stats: epilogue partial slabs come back raw, (R, B, C); the fold sums their slots and
                # takes |.| for Taylor in its one launch (|.| of the already-final slabs is a no-op)
                take_abs = stats and mode == "taylor"
                for i, x, y, lb in self._coalesced_batches(False, big):
                    def fold(res, dev=x.device):
                        slabs = [res[m] for m in uniq]
                        sums = [accs[first[m]].ensure_sum(res[m].shape[-1], dev, m.num_features) for m in uniq]
                        for j in range(0, len(slabs), 16):
                            ops.score_fold_(slabs[j:j + 16], sums[j:j + 16], take_abs, 0)

                    if pipe is not None and pipe.take(x, y, lambda slot, x=x, y=y, lb=lb: eng.grad_scores(
                            x, y, set(uniq), mode, loss_batch=lb, raw_slabs=True), fold):
                        for m in uniq:
                            accs[first[m]].count += x.shape[0]
                        continue
                    with trace_range("tp.forward_backward"):
                        res = eng.grad_scores(x, y, set(uniq), mode, crit, loss_batch=lb, raw_slabs=stats)
                    if stats:
                        slabs = [res[m] for m in uniq]
                        sums = [accs[first[m]].ensure_sum(res[m].shape[-1], x.device, m.num_features) for m in uniq]
                        for j in range(0, len(slabs), 16):
                            ops.score_fold_(slabs[j:j + 16], sums[j:j + 16], take_abs, 0)
                        for m in uniq:
                            accs[first[m]].count += x.shape[0]
                    else:
                        for m in uniq:
                            accs[first[m]].add(res[m][:, :m.num_features].contiguous(), i)
        finally:  # the tuner's in-flight concurrency is reset even if a batch raises
            if pipe is not None:
                pipe.join()
        return [accs[first[m]] for m in eval_modules]

    def _forward_capture_pass(self, eval_modules, on_out):
        """No-grad forward pass calling ``on_out(k, output, batch_index)`` per module."""
        state = {}

        def make_hook(k):
            def hook(_m, _inp, out):
                on_out(k, out, state["idx"])
            return hook

        handles = [m.register_forward_hook(make_hook(k)) for k, m in enumerate(eval_modules)]
        self.set_deterministic()
        try:
            with torch.no_grad(), self._native_ctx():
                for i, x, _y in self._batches():
                    state["idx"] = i
                    with self._autocast():
                        self.model(x)
        finally:
            for h in handles:
                h.remove()
            self.restore_deterministic()

    def run_many(self, modules, find_best_evaluation_module=False, **kwargs):
        """Scores for several modules. Hook-based metrics share ONE pass over the data
        (new API; the reference runs a full pass per module). Returns a list of arrays."""
        return [self.run(m, find_best_evaluation_module=find_best_evaluation_module, **kwargs) for m in modules]

    def _eval_modules(self, modules, find_best_evaluation_module):
        out = []
        for m in modules:
            assert any(isinstance(m, t) for t in SUPPORTED_OUT_PRUNING_MODULES), \
                f"Attributions can be computed only for the following modules {SUPPORTED_OUT_PRUNING_MODULES}"
            out.append(self.find_evaluation_module(m, find_best_evaluation_module=find_best_evaluation_module))
        return out


def _to(t, device):
    if isinstance(t, torch.Tensor):
        return t.to(device, non_blocking=True)
    return t


class _BatchPipeline:
    """Two batches in flight for small batches on the fused engine (stats reductions only).

    A small batch leaves most of the 256 CUs idle in every layer (a few hundred workgroups, each
    latency-bound), and even a full-size batch idles CUs in every kernel's tail and between the
    ~45 dependent launches of a step; consecutive batches run on two HIP streams and their
    kernels co-execute (measured on MI355X, VGG16 Taylor: B=100 +33%, B=256 +16%, B=2048 +3%).
    ``launch(slot)`` enqueues one batch's engine work into stream-private buffers (slot 0 / 1)
    and returns them; ``fold(buffers)`` folds them into the fp64 sums. The folds are chained by
    an event in batch order, so the accumulated scores are bit-identical to the sequential loop.
    The first batch of every new shape runs alone on the current stream (kernel autotuning,
    buffer allocation, lazily packed operands). Two batches' activations are live at once, so it
    is off for inputs of >= 2^24 pixels per batch (B >= 16384 at 32x32, B >= 335 at 224x224;
    TORCHPRUNER_STREAMS_MAX_PIXELS overrides), with TORCHPRUNER_GRAPHS=1/all (one graph-replayed
    batch at a time), and with TORCHPRUNER_STREAMS=0. ResNet-50 at B=256: APoZ +8%, Taylor +7%
    (round 4, F(2x2) 3x3 kernels); with the F(4x4) band kernels three batches in flight for
    large images (>= 112 x 112: ~70 launches per step, many of them short 7/14-px layers) measured
    +1-2% over two (APoZ 14.96k -> 15.08k, Taylor 7.72k -> 7.87k), while the 32x32 headline
    keeps two (three: -0.6 to -1%).
    On the fused VGG/MLP engine a pipelined batch replays a HIP graph of its step per slot
    (FusedChainEngine.graphs_enabled), captured on the slot's first batch: with two batches in
    flight the B=100 step is host-bound otherwise."""

    MAX_PIXELS = 1 << 24
    DEEP_MAX_PIXELS = 1 << 18  # four in flight up to B=256 at 32x32 (B=512 even, B=1024 / 2048 -4%)

    def __init__(self, engine, graph_replay: bool = False):
        self.engine = engine
        self.graph_replay = graph_replay  # the caller's launch() replays graphs when graphs_enabled(B, True)
        self.enabled = os.environ.get("TORCHPRUNER_STREAMS", "1") != "0"
        self.max_pixels = int(os.environ.get("TORCHPRUNER_STREAMS_MAX_PIXELS", self.MAX_PIXELS))
        # batches in flight: 4 when the batches replay graphs and are small (host-light: B=100
        # +10-19% over 2, B=256 +4%, profiles/bench/pipeline_depth_graphs.txt; at B=2048 four cost
        # 4%, profiles/bench/large_batch_graphs_vs_eager.txt), else 2
        env_depth = os.environ.get("TORCHPRUNER_STREAMS_DEPTH")
        self.depth = max(2, int(env_depth)) if env_depth else None
        self.streams = None
        self.seen = set()
        self.n = 0
        self.fold_done = None  # event: the previous pipelined batch's fold

    def take(self, x, y, launch, fold) -> bool:
        """Run batch (x, y) pipelined and return True, or return False (caller runs it)."""
        graphs = getattr(self.engine, "graphs_enabled", None)
        if not self.enabled or not x.is_cuda or x.shape[0] * math.prod(x.shape[2:]) >= self.max_pixels or \
                (graphs is not None and graphs(x.shape[0]) and os.environ.get("TORCHPRUNER_GRAPHS") in ("1", "all")):
            return False
        key = (tuple(x.shape), tuple(y.shape) if y is not None else None)
        if key not in self.seen:  # autotune / allocate alone, after everything in flight
            self.join()
            self.seen.add(key)
            # this batch's kernel choices are timed as they will run: ``depth`` in flight
            from ..engine.fused_chain import TUNER
            TUNER.concurrency = self._depth_for(x, graphs) if self._depth_for(x, graphs) > 2 else 1
            self._tuning = True
            return False
        self._end_tuning()
        if self.streams is None:
            if self.depth is None:
                self.depth = self._depth_for(x, graphs)
            self.streams = [torch.cuda.Stream(x.device) for _ in range(self.depth)]
        cur = torch.cuda.current_stream(x.device)
        slot = self.n % self.depth
        st = self.streams[slot]
        st.wait_stream(cur)  # the batch's copy (and everything before this run) is done
        with torch.cuda.stream(st):
            bufs = launch(slot)
            if self.fold_done is not None:
                st.wait_event(self.fold_done)
            fold(bufs)
            self.fold_done = torch.cuda.Event()
            self.fold_done.record(st)
        for t in (x, y):
            if t is not None:
                t.record_stream(st)
        self.n += 1
        return True

    def _depth_for(self, x, graphs) -> int:
        if self.depth is not None:
            return self.depth
        small = x.shape[0] * math.prod(x.shape[2:]) <= self.DEEP_MAX_PIXELS
        if small and self.graph_replay and graphs is not None and graphs(x.shape[0], pipelined=True):
            return 4
        return 3 if x.dim() == 4 and x.shape[2] * x.shape[3] >= 112 * 112 else 2

    def _end_tuning(self):
        if getattr(self, "_tuning", False):
            from ..engine.fused_chain import TUNER
            TUNER.concurrency = 1
            self._tuning = False

    def join(self):
        self._end_tuning()
        if self.streams is not None:
            cur = torch.cuda.current_stream(self.streams[0].device)
            for st in self.streams:
                cur.wait_stream(st)
