"""Failure injection for data-parallel attribution (SURVEY.md §5 "Failure detection"): a rank is
killed mid-run (``os._exit``: no cleanup, no final checkpoint), the surviving rank's collective
fails instead of hanging, and a relaunch of the job with the same per-rank checkpoints resumes —
every rank recomputes only the batches it had not checkpointed — and returns exactly the scores
of an uninterrupted single-process run (gloo, world 2, CPU)."""
import datetime
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

N_BATCHES, KILL_AT = 10, 3  # rank 1 dies when it reaches its 3rd owned batch (batch 5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class KillableLoader:
    """DeviceLoader-like; ``shard`` can kill the process on one rank."""

    def __init__(self, x, y, bs, kill_rank=None):
        from torchpruner_amd.data import DeviceLoader
        self.inner = DeviceLoader(x, y, bs)
        self.dataset = self.inner.dataset
        self.kill_rank = kill_rank

    def __len__(self):
        return len(self.inner)

    def __iter__(self):
        return iter(self.inner)

    def shard(self, rank, world):
        for k, (i, x, y) in enumerate(self.inner.shard(rank, world)):
            if self.kill_rank == rank and k == KILL_AT - 1:
                os._exit(17)  # hard kill: no finally blocks, no checkpoint flush
            yield i, x, y


def _setup():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(6, 16), nn.ReLU(), nn.Linear(16, 16), nn.ReLU(), nn.Linear(16, 3)).eval()
    g = torch.Generator().manual_seed(1)
    x, y = torch.randn(N_BATCHES * 4, 6, generator=g), torch.randint(0, 3, (N_BATCHES * 4,), generator=g)
    return model, x, y


def _worker(rank, world, port, ckpt, out, kill):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from torchpruner_amd import TaylorAttributionMetric
    torch.set_num_threads(1)
    model, x, y = _setup()
    dl = KillableLoader(x, y, 4, kill_rank=1 if kill else None)
    computed = []  # batches that actually ran forward on this rank
    model[0].register_forward_hook(lambda mod, i, o: computed.append(o.shape[0]))
    m = TaylorAttributionMetric(model, dl, F.cross_entropy, "cpu", reduction="none", checkpoint=ckpt,
                                checkpoint_every=1)
    res = m.run(model[2], find_best_evaluation_module=True)
    if rank == 0:
        np.save(out, res)
    with open(f"{out}.computed.rank{rank}", "w") as f:
        json.dump(len(computed), f)
    dist.destroy_process_group()


def test_dp_attribution_survives_rank_kill(tmp_path):
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    model, x, y = _setup()
    ref = TaylorAttributionMetric(model, DeviceLoader(x, y, 4), F.cross_entropy, "cpu",
                                  reduction="none").run(model[2], find_best_evaluation_module=True)
    ckpt, out = str(tmp_path / "attr.ckpt"), str(tmp_path / "scores.npy")
    with pytest.raises(Exception):  # rank 1 killed; rank 0's all-gather must fail, not hang
        mp.spawn(_worker, args=(2, _free_port(), ckpt, out, True), nprocs=2, join=True)
    assert not os.path.exists(out)
    assert os.path.exists(ckpt + ".rank1")  # rank 1 checkpointed before it died
    done1 = torch.load(ckpt + ".rank1", weights_only=True)["done"]
    assert done1 == [1, 3]  # its batches before the kill (batch 5 never finished)
    mp.spawn(_worker, args=(2, _free_port(), ckpt, out, False), nprocs=2, join=True)
    got = np.load(out)
    # the relaunch recomputed only the unfinished batches: rank 1 had checkpointed 1 and 3 of its
    # 1, 3, 5, 7, 9; rank 0 (killed by the failed collective after all its batches) had all five
    assert json.load(open(out + ".computed.rank1")) == 3
    assert json.load(open(out + ".computed.rank0")) == 0
    assert got.shape == ref.shape == (N_BATCHES * 4, 16)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)
