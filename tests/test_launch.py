"""The single-node launcher behind ``bench.py --gpus N`` (torchpruner_amd/parallel/launch.py):
N fresh rank processes with torchrun-style env, worst return code propagated, survivors of a
failed rank terminated, no re-spawn under an existing launcher; and bench.py's own use of it
(a child that finds fewer GPUs than ranks exits non-zero). CPU-only (gloo)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from torchpruner_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device="cpu")
    fail = int(os.environ.get("FAIL_RANK", "-1"))
    if ctx.rank == fail:
        sys.exit(7)
    t = torch.tensor([float(ctx.rank + 1)])
    pdist.all_reduce_sum_(t)   # a failed rank leaves the others blocked here
    model = torch.nn.Linear(3, 2)
    torch.manual_seed(ctx.rank)  # deliberately different per rank
    model.weight.data.normal_()
    sync = pdist.sync_module(model)
    if ctx.rank == 0:
        print(json.dumps({{"world_size_seen": dist.get_world_size(), "backend": dist.get_backend(),
                          "sum": float(t.item()), "agreed_before": sync["agreed_before"],
                          "env": [os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")]}}),
              flush=True)
    dist.destroy_process_group()
""")

PARENT = textwrap.dedent("""
    import importlib.util, os, sys
    spec = importlib.util.spec_from_file_location("launch", {path!r})
    launch = importlib.util.module_from_spec(spec); spec.loader.exec_module(launch)
    rc = launch.maybe_spawn(int(sys.argv[1]), {script!r}, [], grace=float(sys.argv[2]))
    assert "torch" not in sys.modules, "the spawning parent must not import torch"
    print("PARENT_RC", rc, flush=True)
    sys.exit(0 if rc is None else rc)
""")


def _run_parent(tmp_path, world, grace=30.0, **env):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(root=ROOT))
    parent = tmp_path / "parent.py"
    parent.write_text(PARENT.format(path=os.path.join(ROOT, "torchpruner_amd", "parallel", "launch.py"),
                                    script=str(script)))
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, str(parent), str(world), str(grace)], env=e, capture_output=True,
                          text=True, timeout=120)


def test_spawn_two_ranks(tmp_path):
    p = _run_parent(tmp_path, 2)
    assert p.returncode == 0, p.stdout + p.stderr
    line = next(ln for ln in p.stdout.splitlines() if ln.startswith("{"))
    out = json.loads(line)
    assert out["world_size_seen"] == 2 and out["backend"] == "gloo"
    assert out["sum"] == 3.0  # 1 + 2: both ranks took part
    assert out["agreed_before"] is False  # per-rank weights detected, then synced (asserted inside)
    assert out["env"] == ["0", "0", "2", "127.0.0.1"]
    assert "PARENT_RC 0" in p.stdout


def test_failed_rank_propagates_and_survivors_are_stopped(tmp_path):
    p = _run_parent(tmp_path, 2, grace=2.0, FAIL_RANK="1")
    assert p.returncode == 7, p.stdout + p.stderr
    assert "rank(s) [1] failed" in p.stderr


def test_no_respawn_under_a_launcher(tmp_path):
    p = _run_parent(tmp_path, 2, RANK="0", WORLD_SIZE="1")
    assert p.returncode == 0 and "PARENT_RC None" in p.stdout, p.stdout + p.stderr


def test_worst_rc():
    sys.path.insert(0, os.path.join(ROOT, "torchpruner_amd", "parallel"))
    try:
        import launch
    finally:
        sys.path.pop(0)
    assert launch._worst([0, 0]) == 0
    assert launch._worst([0, 3, 5]) == 3
    assert launch._worst([-9, 0]) == 137
    assert launch.under_launcher({"RANK": "0", "WORLD_SIZE": "8"})
    assert not launch.under_launcher({})


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py --gpus 2 on a box with fewer GPUs (here: none): the spawned ranks exit 3 with a
    clear message and the parent returns that code."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("box has >= 2 GPUs")
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                          "TORCHPRUNER_SHARE_GPU")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=e, capture_output=True,
                       text=True, timeout=180, cwd=ROOT)
    assert p.returncode == 3, p.stdout + p.stderr
    assert "GPU(s) visible" in p.stderr
