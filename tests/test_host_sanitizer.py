"""Host-side launcher validation under AddressSanitizer + UBSan (SURVEY.md §5 sanitizers).

Builds csrc/tests/launcher_validation.cpp with the kernel launchers (host code instrumented,
device code unchanged) and runs it on the CPU: invalid shapes must be rejected before any GPU
work and the host geometry helpers must be memory-clean."""
import os
import subprocess

import pytest


@pytest.mark.skipif(not os.path.exists(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")), reason="needs hipcc")
def test_launcher_validation_asan():
    from torchpruner_amd._build import build_host_sanitizer
    exe = build_host_sanitizer()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "launcher validation ok" in r.stdout
