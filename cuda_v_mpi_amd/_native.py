"""Loader for the in-tree native extension ``_miint`` (HIP kernels + C++ runtime + RCCL).

The extension is built by ``make ext`` (``__graft_entry__.build()`` does this) into this
package directory so that it travels with the repository snapshot and is what every GPU
test and the benchmark actually load. There is deliberately **no** Python fallback for the
GPU kernels: if the extension is missing and cannot be built, :func:`native` raises loudly.
A missing extension is built on first import; a stale one (older than its sources) is loaded
with a warning unless ``MIINT_AUTOBUILD=1`` (never rebuild behind a profiler's back).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
import threading

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_PKG_DIR)
_lock = threading.Lock()
_mod = None


def extension_path() -> str:
    return os.path.join(_PKG_DIR, "_miint" + sysconfig.get_config_var("EXT_SUFFIX"))


def _sources() -> list[str]:
    pats = ["csrc/kernels/*.hip", "csrc/runtime/*.cpp", "csrc/python/*.cpp",
            "csrc/include/miint/*.hpp"]
    out: list[str] = []
    for p in pats:
        out.extend(glob.glob(os.path.join(_REPO, p)))
    return out


def is_stale() -> bool:
    so = extension_path()
    if not os.path.exists(so):
        return True
    t = os.path.getmtime(so)
    return any(os.path.getmtime(s) > t for s in _sources())


def build(jobs: int = 8, quiet: bool = True) -> str:
    """Compile the extension in-tree with hipcc (gfx950). Returns the .so path."""
    cmd = ["make", "-C", _REPO, f"-j{jobs}", "ext"]
    res = subprocess.run(cmd, capture_output=quiet, text=True)
    if res.returncode != 0:
        msg = (res.stdout or "") + (res.stderr or "")
        raise RuntimeError(f"native build failed ({' '.join(cmd)}):\n{msg[-4000:]}")
    return extension_path()


def native(auto_build: bool = True):
    """Import and return the native module, building it first if needed."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        so = extension_path()
        if auto_build and os.environ.get("MIINT_NO_AUTOBUILD") != "1":
            if not os.path.exists(so):
                if "rocprofiler" in os.environ.get("LD_PRELOAD", ""):
                    # under a profiler preload every child process initialises the GPU,
                    # and `make` / `sh` exec'ing from it is refused on the GPU pool
                    raise ImportError(f"miint native extension not found at {so}; build it "
                                      "(make ext) before profiling")
                build()
            elif is_stale():
                if os.environ.get("MIINT_AUTOBUILD") == "1":
                    build()
                else:  # load what is there (a fresh box may reorder mtimes), but say so
                    print(f"miint: warning: {so} is older than its sources; run `make ext` "
                          "(MIINT_AUTOBUILD=1 rebuilds automatically)", file=sys.stderr)
        if not os.path.exists(so):
            raise ImportError(
                f"miint native extension not found at {so}; run `make ext` in {_REPO}")
        # torch (if used) must be imported first so the HIP runtime is shared.
        if "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except Exception:  # pragma: no cover - torch is optional for the native path
                pass
        from . import _miint  # type: ignore[attr-defined]

        _mod = _miint
        return _mod


def require_gpu() -> int:
    """Number of visible GPUs; raises if there are none (GPU-only entry points)."""
    n = native().device_count()
    if n < 1:
        raise RuntimeError("no HIP device visible: this entry point needs an MI355X (gfx950)")
    return n
