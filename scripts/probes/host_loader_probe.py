"""Host DataLoader cost on the GPU box (parent process with the HIP runtime initialised, as in
bench.py): time to the first batch (worker start) and per batch, for the reference's per-sample
collate and a BatchSampler, num_workers 0 / 1, pin_memory on; then the same loaders feeding
TaylorAttributionMetric.run_many on the fused engine (B=100, 200 batches, random-init VGG16)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def loaders(ds, sb):
    for kind in ("batched", "per_sample"):
        for nw in (0, 1, 4):
            if kind == "per_sample":
                yield kind, nw, torch.utils.data.DataLoader(ds, batch_size=sb, num_workers=nw, pin_memory=True)
            else:
                bs = torch.utils.data.BatchSampler(torch.utils.data.SequentialSampler(ds), sb, drop_last=False)
                yield kind, nw, torch.utils.data.DataLoader(ds, sampler=bs, batch_size=None, num_workers=nw,
                                                            pin_memory=True)


def main():
    import torch.nn.functional as F

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.models import prunable_vgg16
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    sb, n = 100, 200
    ds = torch.utils.data.TensorDataset(torch.randn(n * sb, 3, 32, 32), torch.randint(0, 10, (n * sb,)))
    for kind, nw, dl in loaders(ds, sb):
        t0 = time.perf_counter()
        it = iter(dl)
        next(it)
        t1 = time.perf_counter()
        for _ in it:
            pass
        t2 = time.perf_counter()
        print(f"{kind:10s} workers={nw}: first batch {1e3 * (t1 - t0):8.1f} ms, then {1e3 * (t2 - t1) / (n - 1):6.2f} "
              f"ms/batch ({(n - 1) * sb / (t2 - t1):9.0f} img/s)", flush=True)
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    for kind, nw, dl in loaders(ds, sb):
        TaylorAttributionMetric(model, dl, F.cross_entropy, dev).run_many(convs, True)  # warm / tune
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = TaylorAttributionMetric(model, dl, F.cross_entropy, dev)
        m.run_many(convs, True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"run_many {kind:10s} workers={nw}: {n * sb / dt:9.0f} img/s ({m.last_path['path']}, coalesce "
              f"{m.last_coalesce})", flush=True)


if __name__ == "__main__":
    main()
