"""Where the time goes in run_many over a worker-backed host DataLoader (B=100, VGG16 Taylor):
time inside the loader's __next__ vs outside, per batch."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


class Timed:
    def __init__(self, dl):
        self.dl, self.t_in, self.n, self.gaps = dl, 0.0, 0, []

    def __len__(self):
        return len(self.dl)

    def __iter__(self):
        it = iter(self.dl)
        last = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            self.gaps.append(t0 - last)
            try:
                b = next(it)
            except StopIteration:
                return
            t1 = time.perf_counter()
            self.t_in += t1 - t0
            self.n += 1
            last = t1
            yield b


def main():
    import torch.nn.functional as F

    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.models import prunable_vgg16
    dev = torch.device("cuda")
    sb, n = 100, 200
    ds = torch.utils.data.TensorDataset(torch.randn(n * sb, 3, 32, 32), torch.randint(0, 10, (n * sb,)))
    model = prunable_vgg16().to(dev).eval()
    convs = [m for m in model.features if isinstance(m, torch.nn.Conv2d)]
    for nw in (1, 0):
        bs = torch.utils.data.BatchSampler(torch.utils.data.SequentialSampler(ds), sb, drop_last=False)
        dl = torch.utils.data.DataLoader(ds, sampler=bs, batch_size=None, num_workers=nw, pin_memory=True)
        TaylorAttributionMetric(model, dl, F.cross_entropy, dev).run_many(convs, True)
        td = Timed(dl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        TaylorAttributionMetric(model, td, F.cross_entropy, dev).run_many(convs, True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        g = sorted(td.gaps[1:])
        print(f"workers={nw}: {n * sb / dt:8.0f} img/s; {td.n} batches, in next() {1e3 * td.t_in:7.1f} ms of "
              f"{1e3 * dt:7.1f}; gap outside next() median {1e3 * g[len(g) // 2]:.2f} ms max {1e3 * g[-1]:.2f} ms; "
              f"largest 5 gaps {[round(1e3 * x, 1) for x in g[-5:]]}", flush=True)


if __name__ == "__main__":
    main()
