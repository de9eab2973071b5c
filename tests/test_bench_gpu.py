"""``python bench.py --gpus 2`` on the one-GPU box: bench.py spawns its own two rank processes
(no torchrun; the parent process never touches the GPU), both ranks share the MI355X
(``TORCHPRUNER_SHARE_GPU=1``) over gloo, and rank 0's JSON line reports n_gpus 2 and the world
size the process group actually saw. Small config (B=64, 2 steps, short teacher): this checks
the launch / sharding / reporting path, not the throughput."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_two_ranks(cuda):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TORCHPRUNER_SHARE_GPU="1", TORCHPRUNER_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--batch", "64", "--teacher-steps", "20", "--no-baseline", "--no-prune", "--no-extras"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size_seen"] == 2, out
    assert out["dist_backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 128
    assert out["teacher_sync"]["agreed_before_broadcast"] is True  # deterministic native training
    assert out["value"] > 0
