"""The per-sample fp64 sin / cos of the kIeee Sin and TrainVel tiles (fast_trig.hpp), run on
the host (the same __host__ __device__ functions, contraction off) against long double
sinl / cosl. The reference's per-sample form is cintegrate.cu:66-70 / riemann.cpp:37."""
from __future__ import annotations

import math

import pytest
import torch

from cuda_v_mpi_amd import native


def _fast(x: torch.Tensor, shift: int):
    x = x.to(torch.float64).contiguous()
    v, e = torch.empty_like(x), torch.empty_like(x)
    native().fast_trig_host(x.data_ptr(), x.numel(), shift, v.data_ptr(), e.data_ptr())
    return v, e


CASES = {
    "dense_0_pi": lambda: torch.linspace(0.0, math.pi, 1_000_001, dtype=torch.float64),
    "random_1e5": lambda: torch.empty(1_000_000, dtype=torch.float64).uniform_(
        -1e5, 1e5, generator=torch.Generator().manual_seed(3)),
    "dense_at_1e5": lambda: 1e5 + torch.arange(500_000, dtype=torch.float64) * 1e-9,
    "below_pi": lambda: math.pi - torch.arange(1, 200_001, dtype=torch.float64) * 3.14e-9,
    "quadrant_edges": lambda: torch.cat([k * math.pi / 4 + torch.linspace(-1e-6, 1e-6, 20_001,
                                                                          dtype=torch.float64)
                                         for k in range(1, 16, 2)]),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("shift", [0, 1])
def test_fast_trig_within_one_ulp_of_true(case, shift):
    """< 0.9 ulp of the true sin / cos everywhere (fdlibm kernels with the Cody-Waite tail),
    correctly rounded for >= 90 % of the samples (97 % away from the pi/4 quadrant edges)."""
    v, e = _fast(CASES[case](), shift)
    ok = ~torch.isnan(e)
    assert ok.double().mean() > 0.999  # the fast path takes (almost) every sample
    ea = e[ok].abs()
    assert float(ea.max()) < 0.9
    assert float((ea <= 0.5).double().mean()) > (0.9 if case == "quadrant_edges" else 0.96)


def test_fast_trig_declines_where_it_must():
    """Beyond |n| = 65536 quadrants (|x| ~ 1.03e5) the tile hands over to the library (the
    host form returns NaN there), and right at a zero of sin/cos it does so exactly when the
    reduced angle falls below |n P2| (Fast2Sum's precondition); the samples it keeps there
    are still within 1 ulp of the (tiny) true value."""
    f64 = dict(dtype=torch.float64)
    v, _ = _fast(torch.tensor([2e5, -3e5, 1e300, float("inf"), float("nan")], **f64), 0)
    assert torch.isnan(v).all()
    x0 = 1000 * math.pi / 2  # the doubles around 500 pi: sin ~ 1e-13
    xs = [x0]
    lo = hi = x0
    for _ in range(8):
        lo, hi = math.nextafter(lo, -math.inf), math.nextafter(hi, math.inf)
        xs = [lo] + xs + [hi]
    v, e = _fast(torch.tensor(xs, **f64), 0)
    kept = ~torch.isnan(v)
    assert 0 < int(kept.sum()) < len(xs)  # one side of the zero declined, the other kept
    assert float(e[kept].abs().max()) < 1.0
    v, e = _fast(torch.tensor([0.0, 1e-300, 0.5, 1.0, -2.0], **f64), 0)
    assert v[0] == 0.0 and v[1] == 1e-300 and float(e.abs().max()) <= 0.5
