"""1 - APoZ (Average Percentage of Zeros) — Hu et al. (reference: methods/apoz.py:6-39).

Per sample and unit: count of positive outputs summed over the trailing (spatial) dims. For
convolutions this is a *count*, not a fraction, exactly like the reference (apoz.py:31-33).
The count is produced on device by the HIP channel-reduction kernel and accumulated in fp64;
the pass is forward-only and skips the loss the reference computes but never uses.
"""
from ... import ops
from ..base import _AttributionMetric


class APoZAttributionMetric(_AttributionMetric):
    def run(self, module, **kwargs):
        module = super().run(module, **kwargs)
        return self._run_modules([module])[0]

    def run_many(self, modules, find_best_evaluation_module=False, **kwargs):
        return self._run_modules(self._eval_modules(modules, find_best_evaluation_module))

    def _run_modules(self, eval_modules):
        accs = [self._new_accumulator() for _ in eval_modules]
        self._begin_run(accs, eval_modules)
        try:
            self._forward_capture_pass(eval_modules,
                                       lambda k, out, i: accs[k].add(ops.channel_reduce(out, None, "apoz"), i))
        finally:
            self._end_run()
        return [self._finalize(a) for a in accs]
