"""First-order Taylor expansion — Molchanov et al. (reference: methods/taylor.py:6-49).

Per sample: |sum over trailing dims of -(dL/dz * z)| (no abs with ``signed=True``).
The activation and gradient are read once by one fused HIP reduction; the reference keeps a
full activation clone per batch and leaks it on the module (taylor.py:35).
"""
from ... import ops
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
        why = []
        fused = self._fused_engine(eval_modules, why, need_ce=False)  # any criterion (autograd on the logits)
        rn = None if fused is not None else self._resnet_grad_engine(eval_modules, why)
        self._record_path("fused" if fused else "resnet" if rn else "generic", eval_modules, why)
        if fused is not None:
            # native path: one fused forward + input-grad backward scores every module, then
            # ONE fold launch turns all layers' per-sample sums into |.| and fp64 accumulators
            accs = self._fused_grad_pass(*fused, accs, "taylor", not self.signed)
        elif rn is not None:
            accs = self._resnet_grad_pass(rn, eval_modules, accs, mode)
        else:
            self._grad_capture_pass(eval_modules,
                                    lambda k, a, g, i: accs[k].add(ops.channel_reduce(a, g, mode), i))
        return [self._finalize(a) for a in accs]
