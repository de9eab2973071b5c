"""Data-parallel attribution on the native HIP engines with more than one rank (GPU).

Spawns 2 and 3 rank processes (3 = a ragged split of the 7 batches) of tests/dist_gpu_worker.py
on the one leased MI355X: gloo collectives, ranks sharing the device (TORCHPRUNER_SHARE_GPU=1).
Each rank checks that the sharded Taylor / Sensitivity / APoZ / Shapley scores of the fused VGG
engine and APoZ / Taylor of the ResNet engine equal the single-rank scores (<= 1e-6 relative,
Shapley <= 1e-5) and that the engines — not the generic hook path — served every run.
The ranks are child processes (no exec from this process); each has its own time limit.
"""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_gpu_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_dp_engines_match_single_rank(cuda, world):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TORCHPRUNER_DIST_BACKEND="gloo", TORCHPRUNER_SHARE_GPU="1",
                   PYTHONUNBUFFERED="1")
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=100)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} failed (rc={p.returncode}):\n{out[-4000:]}"
    print(outs[0])
    assert f"DIST_GPU_OK world={world}" in outs[0]


RCCL_SCRIPT = r"""
import os, torch, torch.distributed as dist
from torchpruner_amd.parallel import dist as pdist
ctx = pdist.init_distributed()
assert ctx.world_size == 1 and ctx.device.type == "cuda"
# world 1 does not create a group by itself: create the RCCL one explicitly (backend "nccl")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=ctx.device)
assert dist.get_backend() == "nccl"
t = torch.arange(8, dtype=torch.float64, device=ctx.device)
dist.all_reduce(t)
out = [torch.empty_like(t)]
dist.all_gather(out, t)
dist.broadcast(t, 0)
dist.barrier()
torch.cuda.synchronize()
assert torch.equal(out[0], torch.arange(8, dtype=torch.float64, device=ctx.device))
dist.destroy_process_group()
print("RCCL_OK", torch.cuda.get_device_name(0))
"""


def test_rccl_collectives_single_rank(cuda):
    """RCCL (the ``nccl`` backend on ROCm) initialises and runs all_reduce / all_gather /
    broadcast / barrier on the box's MI355X (one rank: the pool leases one GPU; multi-GPU RCCL
    runs are the driver's 8-GPU scaling bench)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, "-c", RCCL_SCRIPT], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=100)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "RCCL_OK" in p.stdout

