"""Sensitivity: mean |dL/dz| per unit — Mittal et al. (reference: methods/sensitivity.py:5-34).

Per sample: sum over trailing dims of |grad_output|, gradient of the per-batch *mean* loss
(so scores scale with 1/batch_size, as in the reference).
"""
from ... import ops
from ..base import _AttributionMetric


class SensitivityAttributionMetric(_AttributionMetric):
    def run(self, module, **kwargs):
        module = super().run(module, **kwargs)
        return self._run_modules([module])[0]

    def run_many(self, modules, find_best_evaluation_module=False, **kwargs):
        return self._run_modules(self._eval_modules(modules, find_best_evaluation_module))

    def _run_modules(self, eval_modules):
        accs = [self._new_accumulator() for _ in eval_modules]
        self._begin_run(accs, eval_modules)
        try:
            why = []
            fused = self._fused_engine(eval_modules, why, need_ce=False)  # any criterion (autograd on the logits)
            rn = None if fused is not None else self._resnet_grad_engine(eval_modules, why)
            self._record_path("fused" if fused else "resnet" if rn else "generic", eval_modules, why)
            if fused is not None:  # VGG-style chains: |dL/da| partials from the fused dgrad epilogues
                accs = self._fused_grad_pass(*fused, accs, "sensitivity", False)
            elif rn is not None:  # ResNets: forward + input-grad backward on the HIP engine
                accs = self._resnet_grad_pass(rn, eval_modules, accs, "sensitivity")
            else:
                self._grad_capture_pass(eval_modules,
                                        lambda k, a, g, i: accs[k].add(ops.channel_reduce(None, g, "sensitivity"), i))
        finally:
            self._end_run()
        return [self._finalize(a) for a in accs]
