"""Staged-window kernels under LDS poisoning (native.set_lds_poison): every LDS word a kernel
does not stage reads NaN, so a read past the staged window — which with stale LDS contents
can pass silently — turns the result NaN. Each case compares with a torch fp64 reference of
the same samples.

Covered: the train-scan samplers (trainscan.hip make_sampler; 4main.c:82-86's fill inside
the scan), interp_fill's per-workgroup chunk windows (cintegrate.cu:88-92's fill) and the
2-D row stream's footprint tile (BASELINE #5). The train-scan case is the adversarial one of
commit 7acfd1e: at dt = 1/3007 the hot form's t = fma(k, dt, t_first) of a tile's last
sample rounds up to exactly 1000.0 while dt * i stays below it, moving the sample into the
next segment with weight 0 — whose right end the staging must include (it did not before
7acfd1e: NaN here; profiles/r3/lds_poison_pre_fix.txt shows that run)."""
from __future__ import annotations

import math

import pytest
import torch

from cuda_v_mpi_amd.ops import kernels
from cuda_v_mpi_amd.utils import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture()
def poison(native, cuda):
    native.set_lds_poison(True)
    try:
        yield
    finally:
        native.set_lds_poison(False)


def _interp_ref(n: int, i0: int, dt: float) -> torch.Tensor:
    """torch fp64 samples of the profile at t = dt * i (segment clamped in fp64)."""
    tab = torch.as_tensor(fixtures.profile_table(), dtype=torch.float64, device="cuda")
    i = torch.arange(i0, i0 + n, dtype=torch.float64, device="cuda")
    t = dt * i
    s = torch.clamp(t, 0.0, float(tab.numel() - 2)).floor().long()
    v0 = tab[s]
    return v0 + (tab[s + 1] - v0) * (t - s.double())


def _adversarial_i0() -> tuple[float, int]:
    """dt and the slice start that put a tile's last sample at index 3007 * 1000."""
    dt = 1.0 / 3007
    il = 3007 * 1000
    # the hot form of trainscan.hip's Sampler::items for that sample
    tb = dt * float(il - 15)
    assert dt * float(il) < 1000.0          # its reference t is below the integer ...
    from fractions import Fraction
    hot = Fraction(15) * Fraction(dt) + Fraction(tb)
    assert hot.numerator / hot.denominator >= 1000.0  # ... the hot form's t is not
    return dt, il - 4095  # tile 0 of the slice ends at il


@pytest.mark.parametrize("algo", ["fused", "onepass"])
def test_trainscan_hot_form_crossing_staged(poison, algo):
    dt, i0 = _adversarial_i0()
    n = 4 * 4096 + 123
    vel, pos, totals = kernels.trainscan(n, i0=i0, dt=dt, algo=algo)
    x = _interp_ref(n, i0, dt)
    assert torch.isfinite(vel).all() and torch.isfinite(pos).all()
    torch.testing.assert_close(vel, torch.cumsum(x, 0), rtol=1e-11, atol=1e-7)
    torch.testing.assert_close(pos, torch.cumsum(torch.cumsum(x, 0), 0), rtol=1e-10, atol=1e-3)


@pytest.mark.parametrize("dt,i0", [(1e-4, 0), (1.05e-4, 7), (2e-3, 123), (1.0 / 3007, 3002905),
                                   (0.37, 5)])
def test_trainscan_samplers_poisoned(poison, dt, i0):
    n = 300_001
    vel, pos, _ = kernels.trainscan(n, i0=i0, dt=dt)
    x = _interp_ref(n, i0, dt)
    assert torch.isfinite(vel).all()
    torch.testing.assert_close(vel, torch.cumsum(x, 0), rtol=1e-11, atol=1e-7)


@pytest.mark.parametrize("i0,n,dt", [(0, 18_000_001, 1e-4), (5, 10_001, 0.37),
                                     (3002905, 1_000_003, 1.0 / 3007), (17_999_000, 1001, 1e-4),
                                     (7, 4_000_000, 4.5e-4)])
def test_interp_fill_chunk_windows_poisoned(poison, i0, n, dt):
    got = kernels.interp_fill(n, i0=i0, dt=dt)
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, _interp_ref(n, i0, dt), rtol=0, atol=1e-12)


@pytest.mark.parametrize("g", [4095, 5000, 8191])
@pytest.mark.parametrize("rows", [None, (1, 2048), (333, 4094), (4093, 4095)])
def test_table2d_stream_footprint_poisoned(native, poison, g, rows):
    """The row stream's staged footprint on non-power-of-two grids and odd row slices: tile
    slots outside the computed footprint are NaN, so the sum is finite only if every read
    stays inside it; and it equals the torch fp64 bilinear midpoint sum."""
    v = torch.as_tensor(fixtures.profile_table(), device="cuda")
    T = kernels.outer_product(v)
    r0, r1 = rows if rows is not None else (0, g)
    assert native.table2d_path(1801, 1801, 1800.0, 1800.0, g, g, r0, r1) == "stream"
    got = float(kernels.table2d(T, 1800.0, 1800.0, g, g, r0, r1).item())
    want = kernels.table2d_reference(T, 1800.0, 1800.0, g, g, r0, r1)
    assert math.isfinite(got)
    assert got == pytest.approx(want, rel=1e-12)
