"""Single-node multi-process launcher: one child process per GPU, torchrun-style environment.

``python bench.py --gpus N`` (and any script that calls :func:`maybe_spawn` first) becomes an
N-rank job without ``torchrun``: the parent process never touches the GPU — this module imports
nothing but the standard library, so no HIP runtime is initialised before the children start
(and nothing is exec'd over a GPU-initialised process) — it starts N fresh interpreters with
``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``LOCAL_WORLD_SIZE`` / ``MASTER_ADDR`` /
``MASTER_PORT`` set, streams their output through (rank 0 prints the result line), and exits
with the worst child return code. Under ``torchrun`` (``WORLD_SIZE`` already in the
environment) nothing is spawned.

Failure handling (the SURVEY §5 failure-detection analogue for a single node): when one rank
dies, the others are blocked in a collective that can never complete, so they get ``grace``
seconds to finish on their own and are then terminated (SIGTERM, then SIGKILL). Children get
``PR_SET_PDEATHSIG`` so that a killed parent does not leave ranks holding the GPU.

Elastic restart (``max_restarts``, torchrun's ``--max-restarts`` semantics for one node): after a
failure the whole group is stopped and relaunched on a fresh rendezvous port, up to
``max_restarts`` times; each generation sees ``TORCHELASTIC_RESTART_COUNT`` (the variable torchrun
exports). A job that checkpoints per rank (``_AttributionMetric(checkpoint=...)``,
``checkpoint.save_accumulators``) resumes from its checkpoints and recomputes only unfinished
work, so a transient rank loss costs one relaunch, not the job. The same scripts work unchanged
under ``torchrun --max-restarts N``.

The reference has no launcher or distributed code at all; the loop this
parallelises is the attribution data loop, reference ``torchpruner/attributions/attributions.py:58-68``.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Optional, Sequence

RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()


def under_launcher(env=None) -> bool:
    """True when this process is already one rank of a launched job (torchrun or ours)."""
    env = os.environ if env is None else env
    return "WORLD_SIZE" in env and "RANK" in env


def restart_count(env=None) -> int:
    """Generation of this rank process: 0 on the first launch, k after the k-th elastic restart
    (set by :func:`spawn_local` and by torchrun)."""
    env = os.environ if env is None else env
    return int(env.get("TORCHELASTIC_RESTART_COUNT", "0"))


def rank_env(rank: int, world: int, port: int, base=None, addr: str = "127.0.0.1", restart: int = 0) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR=addr, MASTER_PORT=str(port), PYTHONUNBUFFERED="1",
               TORCHELASTIC_RESTART_COUNT=str(restart))
    # dmabuf IPC only on this platform (RCCL / CUDA-tensor sharing fails without it)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _pdeathsig():  # runs in the child between fork and exec: no GPU state exists in the parent
    try:
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except Exception:
        pass


def _worst(rcs: Sequence[Optional[int]]) -> int:
    """Worst return code: the first non-zero one in rank order (signals as 128+sig), else 0."""
    for rc in rcs:
        if rc is None:
            return 1
        if rc != 0:
            return 128 - rc if rc < 0 else rc
    return 0


def spawn_local(nproc: int, argv: Sequence[str], *, python: str = sys.executable, env: Optional[dict] = None,
                grace: float = 60.0, timeout: Optional[float] = None, cwd: Optional[str] = None,
                log=None, max_restarts: int = 0) -> int:
    """Run ``python argv...`` as ``nproc`` ranks on this node; return the return code of the
    first rank that failed (the root cause; peers blocked in a collective fail after it), 0 if
    none did.

    Children inherit stdout/stderr (rank 0's result line reaches the caller unmodified).
    ``grace``: seconds the surviving ranks get after the first failure; ``timeout``: overall
    limit per generation (None = none); ``max_restarts``: relaunch the whole group this many
    times after a failure (elastic restart, see the module docstring)."""
    assert nproc >= 1 and max_restarts >= 0
    log = log or (lambda msg: print(msg, file=sys.stderr, flush=True))
    for gen in range(max_restarts + 1):
        rc = _run_group(nproc, argv, python, env, grace, timeout, cwd, log, gen)
        if rc == 0:
            return 0
        if gen < max_restarts:
            log(f"[launch] group failed (rc {rc}); elastic restart {gen + 1}/{max_restarts}")
    return rc


def _run_group(nproc, argv, python, env, grace, timeout, cwd, log, gen) -> int:
    port = free_port()
    procs = []
    try:
        for r in range(nproc):
            procs.append(subprocess.Popen([python, *argv], env=rank_env(r, nproc, port, env, restart=gen), cwd=cwd,
                                          preexec_fn=_pdeathsig))
        t0 = time.monotonic()
        failed_at = None
        first_rc = 0
        while True:
            rcs = [p.poll() for p in procs]
            if all(rc is not None for rc in rcs):
                break
            now = time.monotonic()
            if failed_at is None and any(rc not in (None, 0) for rc in rcs):
                failed_at = now
                bad = [r for r, rc in enumerate(rcs) if rc not in (None, 0)]
                first_rc = _worst([rcs[r] for r in bad])  # the root cause, not the peers it took down
                log(f"[launch] rank(s) {bad} failed (rc {[rcs[r] for r in bad]}); stopping the others in {grace:.0f}s")
            if (failed_at is not None and now - failed_at > grace) or (timeout is not None and now - t0 > timeout):
                log("[launch] terminating the remaining ranks")
                _terminate(procs)
                break
            time.sleep(0.2)
    except BaseException:
        _terminate(procs)
        raise
    rcs = [p.wait() for p in procs]
    return first_rc or _worst(rcs)


def _terminate(procs, wait: float = 10.0):
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + wait
    for p in procs:
        try:
            p.wait(max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def maybe_spawn(nproc: int, script: str, args: Sequence[str], **kw) -> Optional[int]:
    """When ``nproc > 1`` and this process is not already a rank, run ``script args`` as
    ``nproc`` ranks and return the worst return code; otherwise return None (run in-process)."""
    if nproc <= 1 or under_launcher():
        return None
    return spawn_local(nproc, [script, *args], **kw)


def main(argv: Optional[Sequence[str]] = None) -> int:
    """``python -m torchpruner_amd.parallel.launch --nproc N [--max-restarts K] script.py args...``:
    a standard-library-only, single-node stand-in for ``torchrun`` (no GPU touched here)."""
    import argparse
    ap = argparse.ArgumentParser(prog="python -m torchpruner_amd.parallel.launch")
    ap.add_argument("--nproc", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--max-restarts", type=int, default=0, help="elastic relaunches of the group after a failure")
    ap.add_argument("--grace", type=float, default=60.0, help="seconds survivors get after a rank fails")
    ap.add_argument("--timeout", type=float, default=None, help="per-generation time limit (seconds)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    return spawn_local(a.nproc, [a.script, *a.args], grace=a.grace, timeout=a.timeout, max_restarts=a.max_restarts)


if __name__ == "__main__":
    sys.exit(main())
