"""In-tree native build for the MI355X (gfx950) extension ``torchpruner_amd/_C.so``.

Design
------
* Every ``csrc/kernels/*.hip`` file is plain HIP (no torch headers) and is compiled
  with ``hipcc --offload-arch=gfx950`` into an object file. Kernel files export
  host-side launcher functions that take raw device pointers + a ``hipStream_t``.
* ``csrc/bindings.cpp`` is the only translation unit that includes torch. It
  validates tensors (device / dtype / contiguity / shape — ops fail loudly on a
  mismatch) and registers the ``torch.ops.tpamd.*`` operators with
  ``TORCH_LIBRARY``.
* Everything is linked with ``-shared`` into ``torchpruner_amd/_C.so`` against the
  HIP runtime that ships inside torch (same soname ``libamdhip64.so.7``), so the
  extension shares torch's streams and caching allocator.

The reference has no native code at all; this replaces the
implicit cuDNN/cuBLAS/ATen kernels its hooks trigger.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD_DIR = ROOT / "build" / "native"
OUT = Path(__file__).resolve().parent / "_C.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    lib = tdir / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _common_flags():
    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-ffp-contract=fast",
        "-munsafe-fp-atomics",
        f"-I{CSRC / 'include'}",
        "-Wno-unused-result",
        # extra flags for experiment builds, e.g. -DTP_WINO_DEBUG (scripts/gpu_wino_epi_attr.sh)
        *os.environ.get("TORCHPRUNER_HIPFLAGS", "").split(),
    ]


# per-file extra flags. wino4: the SLP vectorizer packs the scalar Winograd transforms into
# v_pk_* f32 ops plus operand-shuffling moves (182 v_mov in the main loop, VGPR spills); packed
# f32 VALU also issues slower beside MFMAs than scalar FMAs (MI355X_MICROARCH.md constants table)
FILE_FLAGS = {"wino4": ["-fno-slp-vectorize"]}


def _needs_rebuild(src: Path, obj: Path, deps: list[Path]) -> bool:
    """mtime check (host-sanitizer build only; the extension itself rebuilds by content hash)."""
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"native build failed: {' '.join(str(c) for c in cmd[:6])} ...")
    return r


# ---------------------------------------------------------------- content hashes
# The extension is rebuilt from what the sources SAY, not from file times: an object is recompiled
# when the hash of its source + headers + (path-free) flags differs from the one recorded when it
# was built (build/native/manifest.json), and the hash of the whole source set is stamped into
# _C.so as the string ``TPAMD_SRC_HASH=<hex>``, the hash of the build flags / torch version as
# ``TPAMD_FLAG_HASH=<hex>``. ops.load() refuses a _C.so whose source stamp does not match the tree
# it runs from (a stale binary after a checkout or a copy that refreshed mtimes unevenly would
# otherwise load silently); a flag-stamp mismatch (an env var of the build shell such as
# TORCHPRUNER_HIPFLAGS / PYTORCH_ROCM_ARCH that differs at load time) only warns.
STAMP_RE = re.compile(rb"TPAMD_SRC_HASH=([0-9a-f]{16})")
FLAG_STAMP_RE = re.compile(rb"TPAMD_FLAG_HASH=([0-9a-f]{16})")


def _flag_sig(stem: str, binding: bool) -> str:
    import torch
    flags = [f for f in _common_flags() if not f.startswith("-I")] + FILE_FLAGS.get(stem, [])
    extra = f"torch={torch.__version__}" if binding else ""
    return " ".join(flags) + "|" + extra


def _digest(paths, sig: str) -> str:
    h = hashlib.sha256(sig.encode())
    for p in paths:
        h.update(p.relative_to(ROOT).as_posix().encode() + b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _sources():
    return (sorted((CSRC / "include").glob("*.h")), sorted((CSRC / "kernels").glob("*.hip")),
            sorted(CSRC.glob("*.cpp")))


def source_hash() -> str:
    """Hash of every source and header that goes into ``_C.so`` (content only: independent of
    the environment of the shell that loads it)."""
    headers, kernels, bindings = _sources()
    per = [_digest([s] + headers, "") for s in kernels + bindings]
    return hashlib.sha256("".join(per).encode()).hexdigest()[:16]


def flag_hash() -> str:
    """Hash of the per-file compile flags (env-dependent: arch, TORCHPRUNER_HIPFLAGS, torch)."""
    _, kernels, bindings = _sources()
    sig = [_flag_sig(s.stem, False) for s in kernels] + [_flag_sig(b.stem, True) for b in bindings]
    return hashlib.sha256("\n".join(sig).encode()).hexdigest()[:16]


def stamped_hash(path: Path = OUT, flags: bool = False):
    """The source (``flags=True``: flag) hash stamped into a built extension (None when absent)."""
    if not path.exists():
        return None
    m = (FLAG_STAMP_RE if flags else STAMP_RE).search(path.read_bytes())
    return m.group(1).decode() if m else None


def build(verbose: bool = False, force: bool = False, jobs: int | None = None) -> Path:
    """Compile all HIP kernels + torch bindings into ``torchpruner_amd/_C.so``."""
    inc, lib, abi = _torch_paths()
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    headers, kernels, bindings = _sources()
    man_path = BUILD_DIR / "manifest.json"
    try:
        manifest = json.loads(man_path.read_text()) if man_path.exists() and not force else {}
    except ValueError:
        manifest = {}

    jobs_list = []
    objs = []
    new_manifest = {}
    for src, is_binding in [(k, False) for k in kernels] + [(b, True) for b in bindings]:
        obj = BUILD_DIR / (src.stem + ".o")
        objs.append(obj)
        dig = _digest([src] + headers, _flag_sig(src.stem, is_binding))
        new_manifest[obj.name] = dig
        if force or not obj.exists() or manifest.get(obj.name) != dig:
            if is_binding:
                cmd = [HIPCC, *_common_flags(), f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
                       "-D__HIP_PLATFORM_AMD__=1", *[f"-I{p}" for p in inc], "-c", src, "-o", obj]
            else:
                cmd = [HIPCC, *_common_flags(), *FILE_FLAGS.get(src.stem, []), f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                       "-c", src, "-o", obj]
            jobs_list.append(cmd)

    n = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    man_path.write_text(json.dumps(new_manifest, indent=1, sort_keys=True))

    want, want_flags = source_hash(), flag_hash()
    if force or jobs_list or stamped_hash() != want or stamped_hash(flags=True) != want_flags:
        stamp_src = BUILD_DIR / "src_stamp.cpp"
        stamp_src.write_text("// generated by torchpruner_amd/_build.py: hashes of the sources / flags of this _C.so\n"
                             f'extern "C" __attribute__((used, visibility("default"))) const char tp_src_stamp[] = '
                             f'"TPAMD_SRC_HASH={want}";\n'
                             f'extern "C" __attribute__((used, visibility("default"))) const char tp_flag_stamp[] = '
                             f'"TPAMD_FLAG_HASH={want_flags}";\n')
        stamp_obj = BUILD_DIR / "src_stamp.o"
        _run([HIPCC, "-fPIC", "-O1", "-x", "c++", "-c", stamp_src, "-o", stamp_obj], verbose)
        tmp = OUT.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, stamp_obj,
               f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
               "-lamdhip64", "-o", tmp]
        _run(cmd, verbose)
        os.replace(tmp, OUT)
    assert stamped_hash() == want, "source stamp missing from the linked extension"
    return OUT


SANITIZE_SOURCES = ("wino4", "conv_mfma", "conv_wgrad", "winograd", "batchnorm", "weight_pack")  # longest compile first


def build_host_sanitizer(verbose: bool = False) -> Path:
    """Build ``csrc/tests/launcher_validation.cpp`` against the kernel launchers with
    AddressSanitizer + UBSan on the HOST code only (``-Xarch_host -fsanitize=...``; GPU
    sanitizers are not available on this pool). The program checks, on a CPU-only machine,
    that every launcher rejects unsupported shapes before touching the GPU and that the host
    geometry helpers are memory-clean. Returns the executable path."""
    out_dir = ROOT / "build" / "asan"
    out_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted((CSRC / "include").glob("*.h"))
    san = ["-Xarch_host", "-fsanitize=address,undefined"]
    jobs, objs = [], []
    for name in SANITIZE_SOURCES:
        src, obj = CSRC / "kernels" / f"{name}.hip", out_dir / f"{name}.o"
        objs.append(obj)
        if _needs_rebuild(src, obj, headers):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", f"-I{CSRC / 'include'}", *san,
                         "-c", src, "-o", obj])
    test_src, test_obj = CSRC / "tests" / "launcher_validation.cpp", out_dir / "launcher_validation.o"
    if _needs_rebuild(test_src, test_obj, headers):
        jobs.append([HIPCC, "-O1", "-g", "-std=c++17", *san, "-c", test_src, "-o", test_obj])
    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 4)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    exe = out_dir / "launcher_validation"
    if jobs or not exe.exists():
        _run([HIPCC, f"--offload-arch={ARCH}", "-fsanitize=address,undefined", test_obj, *objs, "-o", exe], verbose)
    return exe


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
    print(OUT)
