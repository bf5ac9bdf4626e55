"""Host emulations of device numerics (CPU only).

The fp32 Pi4 path (csrc/kernels/riemann.hip, Pi4F32::tile_acc) evaluates each 192-sample
tile as s (U + sum e) from an fp32 seed s ~ 1/d(x_m) and fp32 residuals e. This emulates the
tile with numpy float32 arithmetic (at 128 samples, the length it had when this was found): folding s (U + sum e) in fp32 drops the seed's own
correction (U + sum e rounds at ulp(128) = 1.5e-5 while |sum e| ~ U |e_m| ~ 4e-6) and biases
the integral by ~-8e-9 relative, which is what the GPU printed (3.1415926288, |err| 2.5e-8 at
N = 1e9) before the fold moved to fp64 (|err| 1.0e-9 = h, the left rule's truncation).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def _fma32(a, b, c):
    # float32 inputs: the product is exact in float64, so this is one rounding of a*b + c
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


def _tiles(n: int, u: int = 128):
    h = 1.0 / n
    i = np.arange(n // u, dtype=np.float64)
    xm = (i * u + 0.5 * (u - 1)) * h  # left rule, tile midpoints
    x32 = xm.astype(F32)
    one = np.ones_like(x32)
    dm = _fma32(x32, x32, one)
    s = (1.0 / dm.astype(np.float64)).astype(F32)  # v_rcp_f32 stand-in
    s = _fma32(s, _fma32(-dm, s, one), s)          # one Newton step
    em = _fma32(-dm, s, one)
    sum_e = (F32(u) * em).astype(F32)              # symmetric +-k A terms cancel in the sum
    return h, s, sum_e


def test_fp32_tile_fold_bias_and_fp64_fix():
    n = 10**8
    h, s, sum_e = _tiles(n)
    fold32 = (s * (F32(128) + sum_e)).astype(F32).astype(np.float64).sum() * 4 * h
    fold64 = (s.astype(np.float64) * (128.0 + sum_e.astype(np.float64))).sum() * 4 * h
    exact_left = math.pi + 1.0 / n  # left-rule truncation of 4/(1+x^2) on [0, 1] is h
    assert abs(fold64 - exact_left) < 1e-10 * 4
    assert fold32 - exact_left < -5e-9          # the fp32 fold's negative bias
    assert abs(fold32 - exact_left) > 50 * abs(fold64 - exact_left)
