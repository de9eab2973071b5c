"""Probe: when do DDP's gradient buckets become ready inside the native ResNet-50 backward, and how
much all-reduce would stay exposed after it on an 8-GPU xGMI node, per bucket size (VERDICT r5
weak #8: "nothing shows that gradient buckets overlap the native backward").

One rank, RCCL (``nccl``) process group of size 1, ``DistributedDataParallel`` around the
training model with the native kernels switched in (the config #5 step). A comm hook records a
GPU event when the reducer hands over each bucket (= when the bucket's last gradient was produced
on the compute stream) and then runs the stock all-reduce. From the measured ready times the probe
replays an 8-rank ring on one collective stream: bucket k starts at max(ready_k, end of bucket
k-1) and takes ``lat + 2 (N-1)/N * bytes / busbw``; what ends after the last bucket is ready (the
end of the backward's gradient work) is exposed.

    python scripts/probes/ddp_overlap_probe.py [--caps 4,8,16,25,64] [--rounds 0,1] [--batch 128]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402

from torchpruner_amd import Pruner, get_resnet_pruning_graph  # noqa: E402
from torchpruner_amd.engine.train import enable_native_convs  # noqa: E402
from torchpruner_amd.models import resnet50  # noqa: E402


def replay(ready_ms, nbytes, n, busbw_gbs, lat_us):
    end = 0.0
    for r, b in zip(ready_ms, nbytes):
        end = max(end, r) + lat_us * 1e-3 + 2 * (n - 1) / n * b / (busbw_gbs * 1e9) * 1e3
    return max(0.0, end - max(ready_ms)), end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="4,8,16,25,64")
    ap.add_argument("--rounds", default="0,1")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--busbw", default="100,200,300", help="assumed 8-rank all-reduce bus bandwidths, GB/s")
    ap.add_argument("--lat-us", type=float, default=40.0)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    bws = [float(v) for v in a.busbw.split(",")]
    for rounds in [int(r) for r in a.rounds.split(",")]:
        torch.manual_seed(0)
        model = resnet50().to(dev)
        rng = np.random.RandomState(0)
        pruner = Pruner(model, (3, 224, 224), dev)
        for _ in range(rounds):
            for module, cascade in get_resnet_pruning_graph(model):
                n = module.weight.shape[0]
                pruner.prune_model(module, rng.choice(n, int(n * 0.2), replace=False), cascade)
        model = model.to(memory_format=torch.channels_last).train()
        enable_native_convs(model)
        grad_mb = sum(p.numel() for p in model.parameters()) * 4 / 2 ** 20
        x = torch.randn(a.batch, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (a.batch,), device=dev)
        print(f"[ddp_overlap] rounds={rounds} B={a.batch}: {grad_mb:.1f} MB of fp32 gradients", flush=True)
        for cap in [float(c) for c in a.caps.split(",")]:
            ddp = DDP(model, device_ids=[0], bucket_cap_mb=cap)
            marks = []

            def hook(state, bucket):
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                marks.append((ev, bucket.buffer().numel() * bucket.buffer().element_size()))
                return dist.all_reduce(bucket.buffer(), async_op=True).get_future().then(lambda f: f.value()[0])

            ddp.register_comm_hook(None, hook)
            opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, fused=True)
            rows = []
            for it in range(a.steps + 2):
                marks.clear()
                opt.zero_grad(set_to_none=True)
                loss = F.cross_entropy(ddp(x), y)
                b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                b0.record()
                loss.backward()
                b1.record()
                opt.step()
                torch.cuda.synchronize()
                if it >= 2:  # the first iterations rebuild the buckets in ready order
                    rows.append((b0.elapsed_time(b1), [b0.elapsed_time(e) for e, _ in marks], [nb for _, nb in marks]))
            bwd = float(np.median([r[0] for r in rows]))
            ready = np.median(np.array([r[1] for r in rows]), axis=0).tolist()
            nbytes = rows[-1][2]
            lst = " ".join(f"{r:.1f}/{b / 2 ** 20:.1f}" for r, b in zip(ready, nbytes))
            expo = "  ".join(f"{bw:.0f}GB/s: {replay(ready, nbytes, 8, bw, a.lat_us)[0]:.2f}ms" for bw in bws)
            print(f"[ddp_overlap] rounds={rounds} cap={cap:g}MB: backward {bwd:.2f} ms, {len(ready)} buckets "
                  f"(ready ms/MB: {lst}); exposed after the last: {expo}", flush=True)
            del ddp, opt
        del model, x
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
