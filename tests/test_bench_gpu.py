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


@pytest.mark.timeout(260)
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
    # diagnosability: per-phase wall seconds and the per-layer kernel choices of this box
    assert {"teacher", "headline", "total"} <= set(out["phase_wall_s"])
    assert out["tuner_choices"]["headline"], out["tuner_choices"]


@pytest.mark.timeout(320)
def test_bench_config5_two_ranks(cuda):
    """Config #5 in bench.py at 2 self-launched ranks sharing the GPU: the
    ResNet-50 finetune step after a data-parallel prune + PrunableDDP rewrap, and one prune ->
    finetune round Taylor vs Random from one synced teacher (small shapes: this checks the DDP /
    pruning / reporting path, not the numbers)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TORCHPRUNER_SHARE_GPU="1", TORCHPRUNER_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "1", "--batch", "32", "--teacher-steps", "10", "--no-baseline", "--no-prune",
                        "--extras", "finetune,quality5", "--finetune-batch", "8", "--finetune-res", "64",
                        "--finetune-steps", "2", "--q5-res", "64", "--q5-max-steps", "20"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    out = json.loads(lines[-1])
    assert out["resnet50_finetune_img_s"] > 0 and out["resnet50_train_dense_img_s"] > 0
    cfg = out["resnet50_finetune_config"]
    assert cfg["in_sync"] is True and cfg["loss_finite"] is True
    before, after = cfg["params_before_after"]
    assert after < before  # really pruned, DDP rebuilt on the new shapes
    # iterative: two prune -> rewrap -> finetune rounds (momentum sliced twice), each timed
    rounds = cfg["rounds"]
    assert len(rounds) == 2 and all(r["img_s"] > 0 and r["in_sync"] for r in rounds)
    assert before > rounds[0]["params"] > rounds[1]["params"] == after
    q = out["resnet50_prune_finetune"]
    assert q["teacher_agreed_before_broadcast"] is True  # identical deterministic teachers
    assert q["taylor_in_sync"] is True and q["random_in_sync"] is True
    for k in ("taylor_after_prune", "random_after_prune", "taylor_after_finetune", "random_after_finetune"):
        assert 0.0 <= q[k] <= 1.0
