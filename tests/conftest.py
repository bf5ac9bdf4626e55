"""Test configuration.

Markers
  gpu   needs an MI355X (HIP device). The driver runs `-m "not gpu"` on a CPU box and
        `-m gpu` on a GPU box. GPU tests never fall back to CPU paths: they exercise the
        in-tree native extension (cuda_v_mpi_amd/_miint*.so) and fail if it is missing.

The native extension is built on first use if it is missing, so a fresh checkout works on
both boxes (a stale one is loaded with a warning; `make ext` or MIINT_AUTOBUILD=1 rebuilds).
"""
from __future__ import annotations

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires a HIP GPU (MI355X / gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


HAS_GPU = _has_gpu()


def pytest_collection_modifyitems(config, items):
    if HAS_GPU:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    """The native module (built in-tree if missing; a stale one loads with a warning).
    Loads without a GPU too."""
    from cuda_v_mpi_amd._native import native as load

    return load()


@pytest.fixture(scope="session")
def cuda(native):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def slice_tol():
    """Relative tolerance of a G-rank value (rank slices, all-reduced) against the 1-rank one,
    derived on one GPU from the same G slices summed in every order an all-reduce may use
    (tools/slice_sum_spread.py -> profiles/r6/slice_sum_spread.json: 4x the largest spread,
    at least 4 ulp). Bitwise equality is not the contract — the slices move the series tiles'
    seeds and the partial sums — but a value further out is a real error (a slice lost or
    counted twice moves it by ~1/G)."""
    import json
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "profiles", "r6", "slice_sum_spread.json")
    with open(path) as f:
        table = json.load(f)["tolerance_rel_by_g"]
    return lambda g: float(table[str(g)])
