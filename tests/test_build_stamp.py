"""The native extension carries the hash of the sources it was built from, and the loader refuses
a binary that does not match the tree (an mtime-only rebuild check could keep
a stale _C.so)."""
import pytest

from torchpruner_amd import _build
from torchpruner_amd.ops import _native


def test_source_hash_is_content_based(tmp_path, monkeypatch):
    h, f = _build.source_hash(), _build.flag_hash()
    assert len(h) == 16 and len(f) == 16
    # flags are stamped separately (an experiment build with extra flags is a different binary,
    # but the load-time env must not invalidate a correct one: ADVICE r4)
    monkeypatch.setenv("TORCHPRUNER_HIPFLAGS", "-DTP_SOMETHING")
    assert _build.source_hash() == h
    assert _build.flag_hash() != f
    monkeypatch.delenv("TORCHPRUNER_HIPFLAGS")
    assert _build.flag_hash() == f


def test_loader_refuses_a_stale_extension(monkeypatch):
    if not _build.OUT.exists():
        pytest.skip("extension not built")
    assert _build.stamped_hash() == _build.source_hash(), "in-tree _C.so is stale: run __graft_entry__.build()"
    _native._check_stamp()  # matches: no error
    monkeypatch.setattr(_build, "source_hash", lambda: "0" * 16)
    with pytest.raises(RuntimeError, match="stale native extension"):
        _native._check_stamp()


def test_loader_only_warns_on_a_flag_env_mismatch(monkeypatch):
    if not _build.OUT.exists():
        pytest.skip("extension not built")
    monkeypatch.setenv("TORCHPRUNER_HIPFLAGS", "-DTP_LOAD_SHELL_ONLY")
    with pytest.warns(RuntimeWarning, match="other flags"):
        _native._check_stamp()
