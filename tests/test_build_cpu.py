"""CPU checks of the build system (SURVEY C18 / §7.1 layer 1: the reference's Makefile had one
target at -O0 and a rule for a missing source, B17)."""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None,
                    reason="cmake/ninja not available")
def test_cmake_configures_every_target(tmp_path):
    """The CMake/Ninja build describes the same targets as the Makefile, gfx950 only."""
    p = subprocess.run(["cmake", "-S", REPO, "-B", str(tmp_path), "-G", "Ninja"],
                       capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    t = subprocess.run(["ninja", "-C", str(tmp_path), "-t", "targets", "all"],
                       capture_output=True, text=True, timeout=120)
    assert t.returncode == 0, t.stderr
    names = {line.split(":")[0] for line in t.stdout.splitlines()}
    for target in ("riemann", "cintegrate", "trainscan", "miint", "libmiint.a"):
        assert any(n.endswith(target) for n in names), target
    cache = (tmp_path / "CMakeCache.txt").read_text()
    assert re.search(r"CMAKE_HIP_ARCHITECTURES:\w+=gfx950$", cache, re.M)


def test_makefile_is_gfx950_only_and_optimised():
    mk = open(os.path.join(REPO, "Makefile")).read()
    assert "ARCH     ?= gfx950" in mk
    assert "-O3" in mk
    for target in ("ext", "cli", "lib", "asm", "sanitize", "clean"):
        assert re.search(rf"^{target}:", mk, re.M) or re.search(rf"\b{target}\b", mk), target
    # no CUDA, no hipify output, no dual-platform paths anywhere in the native sources
    for root, _, files in os.walk(os.path.join(REPO, "csrc")):
        for f in files:
            src = open(os.path.join(root, f), errors="replace").read()
            assert "cuda_runtime" not in src and "__CUDA_ARCH__" not in src, f
            assert "__HIP_PLATFORM_NVIDIA__" not in src, f
