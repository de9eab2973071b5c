"""First-order Taylor expansion — Molchanov et al. (reference: methods/taylor.py:6-49).

Per sample: |sum over trailing dims of -(dL/dz * z)| (no abs with ``signed=True``).
The activation and gradient are read once by one fused HIP reduction; the reference keeps a
full activation clone per batch and leaks it on the module (taylor.py:35).
"""
from ... import ops
from ...engine import maybe_engine
from ..base import _AttributionMetric


class TaylorAttributionMetric(_AttributionMetric):
    def __init__(self, *args, signed=False, **kwargs):
        super().__init__(*args, **kwargs)
        self.signed = signed

    def run(self, module, **kwargs):
        module = super().run(module, **kwargs)
        return self._run_modules([module])[0]

    def run_many(self, modules, find_best_evaluation_module=False, **kwargs):
        return self._run_modules(self._eval_modules(modules, find_best_evaluation_module))

    def _run_modules(self, eval_modules):
        mode = "taylor_signed" if self.signed else "taylor"
        accs = [self._new_accumulator() for _ in eval_modules]
        self._begin_run(accs, eval_modules)
        try:
            return self._run_loop(eval_modules, accs, mode)
        finally:
            self._end_run()

    def _run_loop(self, eval_modules, accs, mode):
        fused = maybe_engine(self.model, eval_modules, self.criterion, self.device)
        if fused is not None:
            # native path: one fused forward + input-grad backward scores every module, then
            # ONE fold launch turns all layers' per-sample sums into |.| and fp64 accumulators
            engine, blocks = fused
            owner = {}
            for k, b in enumerate(blocks):
                owner.setdefault(b, k)
            uniq = sorted(owner)
            stats = accs[0].mode == "stats"
            for i, x, y in self._batches():
                B = x.shape[0]
                if stats:
                    arena = engine.score_arena(B, uniq, x.device, tuple(x.shape[2:]))
                    engine.taylor(x, y, set(uniq), arena)
                    sums = [accs[owner[b]].ensure_sum(arena[b].shape[-1], x.device, engine.real_width(b))
                            for b in uniq]
                    ops.score_fold_([arena[b] for b in uniq], sums, not self.signed, 2)
                    for b in uniq:
                        accs[owner[b]].count += B
                else:
                    res = engine.taylor(x, y, set(uniq))
                    ops.score_fold_([res[b] for b in uniq], [None] * len(uniq), not self.signed, 1)
                    for b in uniq:
                        accs[owner[b]].add(engine.per_sample(res[b])[:, :engine.real_width(b)], i)
            accs = [accs[owner[b]] for b in blocks]
        elif (rn := self._resnet_grad_engine(eval_modules)) is not None:
            accs = self._resnet_grad_pass(rn, eval_modules, accs, mode)
        else:
            self._grad_capture_pass(eval_modules,
                                    lambda k, a, g, i: accs[k].add(ops.channel_reduce(a, g, mode), i))
        return [self._finalize(a) for a in accs]
