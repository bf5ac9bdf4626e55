"""Host-side ASan + UBSan run of the runtime's CPU code paths (SURVEY §5 race detection /
sanitizers). GPU-side AddressSanitizer and xnack+ are not available on the target pool;
device-side races are covered by the bitwise-determinism GPU tests instead."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_host_selftest_under_asan_ubsan():
    b = subprocess.run(["make", "-C", REPO, "sanitize"], capture_output=True, text=True,
                       timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([os.path.join(REPO, "build", "bin", "host_selftest_asan")],
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "HOST SELFTEST OK" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
