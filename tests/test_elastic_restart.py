"""Elastic restart (SURVEY.md §5 "Failure detection"): the single-node launcher relaunches the
whole rank group after a rank dies (torchrun ``--max-restarts`` semantics, generation number in
``TORCHELASTIC_RESTART_COUNT``), and the relaunched ranks resume from their per-rank attribution
checkpoints — only unfinished batches are recomputed and the scores equal an uninterrupted
single-process run (gloo, world 2, CPU)."""
import json
import os
import sys

import numpy as np
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


def test_launcher_elastic_restart_resumes_from_checkpoints(tmp_path):
    sys.path.insert(0, HERE)
    import elastic_worker as w
    from torchpruner_amd import TaylorAttributionMetric
    from torchpruner_amd.data import DeviceLoader
    from torchpruner_amd.parallel import launch

    model, x, y = w.setup()
    ref = TaylorAttributionMetric(model, DeviceLoader(x, y, 4), F.cross_entropy, "cpu",
                                  reduction="none").run(model[2], find_best_evaluation_module=True)
    msgs = []
    rc = launch.spawn_local(2, [os.path.join(HERE, "elastic_worker.py"), str(tmp_path)], env=_env(), grace=20,
                            timeout=240, max_restarts=1, log=msgs.append)
    assert rc == 0, msgs
    assert any("elastic restart 1/1" in m for m in msgs)
    # generation 0 never finished (rank 1 died, rank 0's collective failed)
    assert not (tmp_path / "computed.gen0.rank1").exists()
    # generation 1: rank 1 had checkpointed batches 1 and 3 of its 1, 3, 5, 7, 9 -> recomputes 3;
    # rank 0 had checkpointed all of its batches before the failed collective -> recomputes none
    assert json.loads((tmp_path / "computed.gen1.rank1").read_text()) == 3
    assert json.loads((tmp_path / "computed.gen1.rank0").read_text()) == 0
    got = np.load(tmp_path / "scores.npy")
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)


def test_launcher_gives_up_after_max_restarts(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\n"
                      "open(os.path.join(sys.argv[1], 'gen' + os.environ['TORCHELASTIC_RESTART_COUNT'] + '.r' "
                      "+ os.environ['RANK']), 'w').close()\n"
                      "sys.exit(5 if os.environ['RANK'] == '1' else 0)\n")
    from torchpruner_amd.parallel import launch
    msgs = []
    rc = launch.spawn_local(2, [str(script), str(tmp_path)], env=_env(), grace=5, max_restarts=2, log=msgs.append)
    assert rc == 5
    assert sorted(p.name for p in tmp_path.glob("gen*")) == [f"gen{g}.r{r}" for g in range(3) for r in range(2)]
    assert launch.restart_count({}) == 0 and launch.restart_count({"TORCHELASTIC_RESTART_COUNT": "2"}) == 2
