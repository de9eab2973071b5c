"""Why run_many on a multi-process host DataLoader is slow: one variable at a time
(pin_memory, the engine's stream pipeline, coalescing, the prefetch side stream), B=100, VGG16."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch.nn.functional as F

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.models import prunable_vgg16
    dev = torch.device("cuda")
    sb, n = 100, 200
    ds = torch.utils.data.TensorDataset(torch.randn(n * sb, 3, 32, 32), torch.randint(0, 10, (n * sb,)))
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    print(f"torch threads {torch.get_num_threads()}, OMP_WAIT_POLICY={os.environ.get('OMP_WAIT_POLICY')}, "
          f"cpus {len(os.sched_getaffinity(0))}", flush=True)
    cases = [("w1 pin", 1, True, {}, None), ("w1 pin threads=1", 1, True, {"_THREADS": "1"}, None),
             ("w1 pin threads=4", 1, True, {"_THREADS": "4"}, None), ("w0 pin", 0, True, {}, None)]
    nt0 = torch.get_num_threads()
    for name, nw, pin, env, ctx in cases:
        torch.set_num_threads(int(env.get("_THREADS", nt0)))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            bs = torch.utils.data.BatchSampler(torch.utils.data.SequentialSampler(ds), sb, drop_last=False)
            dl = torch.utils.data.DataLoader(ds, sampler=bs, batch_size=None, num_workers=nw, pin_memory=pin,
                                             multiprocessing_context=ctx if nw else None)
            TaylorAttributionMetric(model, dl, F.cross_entropy, dev).run_many(convs, True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = TaylorAttributionMetric(model, dl, F.cross_entropy, dev)
            m.run_many(convs, True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"{name:22s}: {n * sb / dt:9.0f} img/s (coalesce {m.last_coalesce})", flush=True)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()
