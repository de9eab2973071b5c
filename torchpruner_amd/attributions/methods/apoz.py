"""1 - APoZ (Average Percentage of Zeros) — Hu et al. (reference: methods/apoz.py:6-39).

Per sample and unit: count of positive outputs summed over the trailing (spatial) dims. For
convolutions this is a *count*, not a fraction, exactly like the reference (apoz.py:31-33).
The count is produced on device by the HIP channel-reduction kernel and accumulated in fp64;
the pass is forward-only and skips the loss the reference computes but never uses.
For torchvision-layout ResNets the whole forward runs on the HIP kernels of the ResNet engine
(engine/resnet_engine.py) with the counts fused into the conv epilogues.
"""
import torch

from ... import ops
from ...engine.resnet_engine import maybe_resnet_engine
from ..base import _AttributionMetric, _BatchPipeline


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
            why = []
            fused = self._fused_engine(eval_modules, why, need_ce=False, pre_act_ok=True)
            eng = None if fused is not None or not self._engines_allowed() else \
                maybe_resnet_engine(self.model, eval_modules, self.device, why=why)
            self._record_path("fused" if fused else "resnet" if eng else "generic", eval_modules, why)
            if fused is not None:
                accs = self._chain_pass(*fused, accs)
            elif eng is not None:
                self._engine_pass(eng, eval_modules, accs)
            else:
                self._forward_capture_pass(eval_modules,
                                           lambda k, out, i: accs[k].add(ops.channel_reduce(out, None, "apoz"), i))
        finally:
            self._end_run()
        return [self._finalize(a) for a in accs]

    def _chain_pass(self, engine, blocks, accs):
        """VGG-style chains: counts fused into the fused engine's forward epilogues (pre-pool
        ReLU outputs), forward stopped at the deepest requested block."""
        owner = {}
        for k, b in enumerate(blocks):
            owner.setdefault(b, k)
        uniq = sorted(owner)
        stats = accs[0].mode == "stats"
        pipe = _BatchPipeline(engine, graph_replay=True) if stats and self._ckpt is None else None
        try:
            with torch.no_grad():
                # small batches coalesced into one launch (per-sample counts: no loss involved)
                for i, x, _y, _lb in self._coalesced_batches(pipe is not None,
                                                             lambda x: engine.max_batch(tuple(x.shape[1:]))):
                    B = x.shape[0]

                    def launch(slot, x=x):
                        if engine.graphs_enabled(x.shape[0], pipelined=True):  # host-bound otherwise
                            return engine.apoz_graphed(x, uniq, slot, warm=True)
                        bufs = {b: torch.zeros(x.shape[0], engine._block_width(b), device=x.device) for b in uniq}
                        engine.forward(x, stop_after=uniq[-1], apoz=bufs)
                        return bufs

                    def fold(bufs, dev=x.device):
                        sums = [accs[owner[b]].ensure_sum(bufs[b].shape[1], dev, engine.real_width(b)) for b in uniq]
                        ops.score_fold_([bufs[b] for b in uniq], sums, False, 0)

                    if pipe is not None and pipe.take(x, None, launch, fold):  # two batches in flight (small B)
                        for b in uniq:
                            accs[owner[b]].count += B
                        continue
                    bufs = {b: torch.zeros(B, engine._block_width(b), device=x.device) for b in uniq}
                    engine.forward(x, stop_after=uniq[-1], apoz=bufs)
                    if stats:
                        sums = [accs[owner[b]].ensure_sum(bufs[b].shape[1], x.device, engine.real_width(b)) for b in uniq]
                        ops.score_fold_([bufs[b] for b in uniq], sums, False, 0)
                        for b in uniq:
                            accs[owner[b]].count += B
                    else:
                        for b in uniq:
                            accs[owner[b]].add(bufs[b][:, :engine.real_width(b)], i)
        finally:  # the tuner's in-flight concurrency is reset even if a batch raises
            if pipe is not None:
                pipe.join()
        return [accs[owner[b]] for b in blocks]

    def _engine_pass(self, eng, eval_modules, accs):
        uniq = list(dict.fromkeys(eval_modules))
        stats = accs[0].mode == "stats"
        arena = None
        pipe = _BatchPipeline(eng) if stats and self._ckpt is None else None
        nf = sum(m.num_features for m in uniq)

        def views(flat, B):
            bufs, off = {}, 0
            for m in uniq:
                bufs[m] = flat[off:off + B * m.num_features].view(B, m.num_features)
                off += B * m.num_features
            return bufs

        try:
            with torch.no_grad():
                # batches past the kernels' descriptor range run in slices
                for i, x, _y, _lb in self._coalesced_batches(False, lambda x: eng.max_batch(tuple(x.shape[1:]))):
                    B = x.shape[0]

                    def launch(slot, x=x):
                        bufs = views(torch.zeros(x.shape[0] * nf, device=x.device), x.shape[0])
                        eng.forward(x, bufs)
                        return bufs

                    def fold(bufs, dev=x.device):
                        sums = [accs[k].ensure_sum(m.num_features, dev) for k, m in enumerate(eval_modules)]
                        ops.score_fold_([bufs[m] for m in eval_modules], sums, False, 0)

                    if pipe is not None and pipe.take(x, None, launch, fold):  # two batches in flight
                        for a in accs:
                            a.count += B
                        continue
                    if arena is None or arena.shape[0] != B * sum(m.num_features for m in uniq) or not stats:
                        arena = torch.zeros(B * sum(m.num_features for m in uniq), device=x.device)
                    else:
                        arena.zero_()
                    bufs, off = {}, 0
                    for m in uniq:
                        bufs[m] = arena[off:off + B * m.num_features].view(B, m.num_features)
                        off += B * m.num_features
                    eng.forward(x, bufs)
                    if stats:  # one fold launch for every module's counts (fp64 column sums)
                        sums = [accs[k].ensure_sum(m.num_features, x.device) for k, m in enumerate(eval_modules)]
                        ops.score_fold_([bufs[m] for m in eval_modules], sums, False, 0)
                        for a in accs:
                            a.count += B
                    else:
                        for k, m in enumerate(eval_modules):
                            accs[k].add(bufs[m], i)
        finally:  # the tuner's in-flight concurrency is reset even if a batch raises
            if pipe is not None:
                pipe.join()
