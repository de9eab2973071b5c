"""One rank of the multi-process data-parallel check of the native HIP engines (launched by
tests/test_dist_gpu.py, one process per rank, torchrun-style env: RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT).

All ranks share the one leased MI355X (``TORCHPRUNER_SHARE_GPU=1``) and talk over gloo
(``TORCHPRUNER_DIST_BACKEND=gloo``; RCCL refuses two ranks on one device). On an 8-GPU node the
same code runs one rank per GPU over RCCL. Every rank computes each metric twice:

* single-rank reference: ``shard_data=False`` -> this rank scores EVERY batch alone, no collective;
* data parallel: whole batches round-robin over ranks, fp64 sums all-reduced once per run (R1),
  per-sample slabs gathered in global order (R2), Shapley prefix work split over ranks with the
  permutations broadcast from rank 0 (R3) and the accumulators all-reduced (R4);

and asserts they agree (<= 1e-6 relative, Shapley <= 1e-5) AND that the native engine served
both (``metric.last_path``). Reference loops being parallelised: attributions.py:58-68,
shapley_values.py:40-61. Exit code 0 = pass; rank 0 prints ``DIST_GPU_OK world=N``.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("TORCHPRUNER_AUTOTUNE", "0")  # same kernel config on every rank (no timing races)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torchpruner_amd import (APoZAttributionMetric, SensitivityAttributionMetric,  # noqa: E402
                             ShapleyAttributionMetric, TaylorAttributionMetric, get_resnet_pruning_graph, ops)
from torchpruner_amd.data import DeviceLoader  # noqa: E402
from torchpruner_amd.models import prunable_vgg16  # noqa: E402
from torchpruner_amd.models.resnet import Bottleneck, ResNet  # noqa: E402
from torchpruner_amd.parallel import dist as pdist  # noqa: E402


def _randomize_bn(model):
    g = torch.Generator().manual_seed(5)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            n = m.num_features
            m.running_mean.copy_((torch.rand(n, generator=g) - 0.5) * 0.4)
            m.running_var.copy_(torch.rand(n, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(n, generator=g) + 0.5)
            m.bias.data.copy_((torch.rand(n, generator=g) - 0.5) * 0.4)


def _close(name, got, ref, rtol, atol):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, f"{name}: shape {got.shape} vs {ref.shape}"
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=atol, err_msg=name)
    return float(np.max(np.abs(got - ref) / (np.abs(ref) + atol))) if ref.size else 0.0


def _both(make, run, path, name, report, rtol=1e-6, atol=1e-9, exact=False):
    """Run one metric single-rank (shard_data=False) and data-parallel; compare (``exact``:
    bit-identical)."""
    if os.environ.get("DIST_WORKER_CPU") == "1":  # dry run of the script logic on a CPU box
        path = "generic-partial" if path == "fused" and "shapley" in name else "generic"
    single = make(False)
    ref = run(single)
    assert single.last_path["path"] == path, f"{name}: single-rank ran {single.last_path}"
    dp = make(None)
    got = run(dp)
    assert dp.last_path["path"] == path, f"{name}: data-parallel ran {dp.last_path}"
    if isinstance(ref, list):
        err = max(_close(f"{name}[{i}]", g, r, rtol, atol) for i, (g, r) in enumerate(zip(got, ref)))
    else:
        err = _close(name, got, ref, rtol, atol)
    if exact:
        pairs = zip(got, ref) if isinstance(ref, list) else [(got, ref)]
        for g_, r_ in pairs:
            assert np.array_equal(np.asarray(g_), np.asarray(r_)), f"{name}: not bit-identical (max rel {err})"
    report[name] = err


def main():
    ctx = pdist.init_distributed()
    world, rank, dev = ctx.world_size, ctx.rank, ctx.device
    assert world > 1
    if os.environ.get("DIST_WORKER_CPU") != "1":
        assert dev.type == "cuda"
        ops.require()
    report = {}

    # ---------------- VGG16-BN on the fused chain engine: 7 batches (last ragged) over `world` ranks
    torch.manual_seed(0)
    vgg = prunable_vgg16().to(dev).eval()
    _randomize_bn(vgg)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(6 * 16 + 9, 3, 32, 32, device=dev, generator=g)
    y = torch.randint(0, 10, (x.shape[0],), device=dev, generator=g)
    dl = DeviceLoader(x, y, 16)
    convs = [m for m in vgg.features if isinstance(m, torch.nn.Conv2d)]
    ce = F.cross_entropy

    _both(lambda s: TaylorAttributionMetric(vgg, dl, ce, dev, shard_data=s),
          lambda m: m.run_many(convs, find_best_evaluation_module=True), "fused", "vgg_taylor_mean", report)
    _both(lambda s: TaylorAttributionMetric(vgg, dl, ce, dev, reduction="none", shard_data=s),
          lambda m: m.run_many(convs[9:], find_best_evaluation_module=True), "fused", "vgg_taylor_none", report)
    _both(lambda s: TaylorAttributionMetric(vgg, dl, ce, dev, signed=True, reduction="sum", shard_data=s),
          lambda m: m.run(convs[4], find_best_evaluation_module=True), "fused", "vgg_taylor_signed_sum", report,
          atol=1e-7)
    _both(lambda s: SensitivityAttributionMetric(vgg, dl, ce, dev, shard_data=s),
          lambda m: m.run_many(convs[::3], find_best_evaluation_module=True), "fused", "vgg_sensitivity", report)
    _both(lambda s: APoZAttributionMetric(vgg, dl, ce, dev, shard_data=s),
          lambda m: m.run_many(convs, find_best_evaluation_module=True), "fused", "vgg_apoz", report)

    def sv(s):
        # 2 batches: world 2 shards whole batches, world 3 splits the prefixes of every batch
        np.random.seed(7)  # rank 0's draw is broadcast (R3); single-rank runs draw the same
        return ShapleyAttributionMetric(vgg, DeviceLoader(x[:32], y[:32], 16), ce, dev, sv_samples=2, shard_data=s)

    # the prefix work is cut on the single-rank K-chunk grid and the deltas are summed unscaled
    # in fp64, so the sharded Shapley values are bit-identical to the single-rank ones
    _both(sv, lambda m: m.run(convs[11], find_best_evaluation_module=True), "fused", "vgg_shapley", report,
          exact=True)

    # a per-rank ShardLoader with fewer batches than ranks: sharded by batches (ranks without a
    # batch contribute zeros); reference = the same single batch on one rank
    from torchpruner_amd.data import ShardLoader

    def sv_shard(s):
        np.random.seed(9)
        if s is False:
            return ShapleyAttributionMetric(vgg, DeviceLoader(x[:16], y[:16], 16), ce, dev, sv_samples=2,
                                            shard_data=False)
        world, rank = pdist.get_world_size(), pdist.get_rank()
        sl = ShardLoader.build(lambda i: (x[:16], y[:16]), 1, 16, rank, world)
        return ShapleyAttributionMetric(vgg, sl, ce, dev, sv_samples=2)

    _both(sv_shard, lambda m: m.run(convs[12], find_best_evaluation_module=True), "fused",
          "vgg_shapley_shardloader", report, exact=True)

    # ---------------- ResNet (bottleneck) on the ResNet engine
    torch.manual_seed(0)
    rn = ResNet(Bottleneck, [1, 2, 1, 1], num_classes=10, width=32).to(dev).eval()
    _randomize_bn(rn)
    xr = torch.randn(5 * 6 + 4, 3, 64, 64, device=dev, generator=g)
    yr = torch.randint(0, 10, (xr.shape[0],), device=dev, generator=g)
    dlr = DeviceLoader(xr, yr, 6)
    mods = [m for m, _ in get_resnet_pruning_graph(rn)]
    _both(lambda s: APoZAttributionMetric(rn, dlr, ce, dev, shard_data=s),
          lambda m: m.run_many(mods, find_best_evaluation_module=True), "resnet", "resnet_apoz", report)
    _both(lambda s: TaylorAttributionMetric(rn, dlr, ce, dev, shard_data=s),
          lambda m: m.run_many(mods, find_best_evaluation_module=True), "resnet", "resnet_taylor", report)
    _both(lambda s: TaylorAttributionMetric(rn, dlr, ce, dev, reduction="none", shard_data=s),
          lambda m: m.run_many(mods[-2:], find_best_evaluation_module=True), "resnet", "resnet_taylor_none",
          report)

    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    if rank == 0:
        print(json.dumps({"world": world, "max_rel_err": report}), flush=True)
        print(f"DIST_GPU_OK world={world}", flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
