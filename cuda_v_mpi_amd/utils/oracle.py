"""Correctness oracles in pure Python/NumPy.

Every value here is computed from the reference's own algorithms and data; the native
module has C++ twins (``_miint.oracle``) which tests cross-check against these.
"""
from __future__ import annotations

import math

import numpy as np

from . import fixtures

PI = math.pi


def left_riemann_pi4_error(n: int) -> float:
    """Truncation error of the left rule for 4/(1+x^2) on [0,1]: (f(0)-f(1)) h / 2 = h."""
    return 1.0 / n


def cintegrate_parity(sp: int = 32, sm: int = 2, accurate: bool = True) -> float:
    """cintegrate.cu cuda_test with SP*SM threads (cintegrate.cu:74-98, 124-138).

    Thread r integrates floor(1800/W) seconds starting at r*floor(1800/W); the host sums the
    W partials. accurate=True sums each thread's samples with NumPy's pairwise sum (the
    reference's sequential fp64 sum adds ~1e-6 of noise at the 6th printed decimal).
    """
    tab = fixtures.profile_table()
    w = sp * sm
    chunk = fixtures.PROFILE_SECONDS // w
    dt = 1.0 / fixtures.STEPS_PER_SEC
    total = 0.0
    for r in range(w):
        i = np.arange(r * chunk * fixtures.STEPS_PER_SEC, (r + 1) * chunk * fixtures.STEPS_PER_SEC)
        y = fixtures.interp(tab, dt * i.astype(np.float64))
        total += float(y.sum()) / fixtures.STEPS_PER_SEC
    return total


def trainscan_parity(p: int) -> tuple[float, float]:
    """4main.c with P ranks: (printed distance, last scanned sum-of-sums element).

    Fill partition by whole seconds (4main.c:76-78), scan partition by elements with the
    residual never scanned (4main.c:90-91), root carry fix-up (4main.c:147-154), printed
    element T-2 (4main.c:241).
    """
    T = fixtures.PROFILE_SECONDS * fixtures.STEPS_PER_SEC
    sub = T // p
    fs = (fixtures.PROFILE_SECONDS // p) * fixtures.STEPS_PER_SEC
    tab = fixtures.profile_table()
    dt = 1.0 / fixtures.STEPS_PER_SEC
    ds = np.zeros(T)
    for q in range(p):
        i = np.arange(q * sub, q * sub + sub)
        vals = fixtures.interp(tab, 0.0 + dt * i.astype(np.float64))
        mask = (i >= q * fs) & (i < q * fs + fs)
        ds[q * sub:q * sub + sub] = np.cumsum(np.where(mask, vals, 0.0))
    for q in range(1, p):
        ds[q * sub:q * sub + sub] += ds[(q - 1) * sub + sub - 1]
    distance = ds[T - 2] / fixtures.STEPS_PER_SEC
    blocks = [float(ds[q * sub:q * sub + sub].sum()) for q in range(p)]
    return float(distance), float(math.fsum(blocks))


def riemann_mpi_parity(comm_size: int, n: float, rng: float = math.pi) -> float:
    """riemann.cpp master/worker (riemann.cpp:65-85): P-1 workers, (int)(n/W) samples each."""
    workers = comm_size - 1
    g = 0.0
    for w in range(workers):
        left = w * (rng / workers)
        right = left + rng / workers
        local_n = int(n / workers)
        h = (right - left) / local_n
        x = left + np.arange(local_n, dtype=np.float64) * h
        g += h * float(np.sin(x).sum())
    return g


def riemann_reference(name: str, n: int, rule: str = "left", a: float | None = None,
                      b: float | None = None, chunk: int = 1 << 22, **kw) -> float:
    """Accurate (pairwise-summed fp64) Riemann sum of a registered integrand, chunked so it
    runs in bounded memory on the CPU."""
    import torch

    from ..models import integrands

    spec = integrands.get(name, **kw)
    a = spec.a if a is None else a
    b = spec.b if b is None else b
    h = (b - a) / n
    off = {"left": 0.0, "mid": 0.5, "right": 1.0}[rule]
    parts = []
    for s in range(0, n, chunk):
        i = torch.arange(s, min(n, s + chunk), dtype=torch.float64)
        parts.append(float(spec.f_torch(a + (i + off) * h).sum()))
    return math.fsum(parts) * h


ORACLES = {
    "pi": PI,
    "sin_0_pi": 2.0,
    "profile_integral": 122000.004000,
    "cintegrate_sp32_sm2": 121999.800663,
    "cintegrate_sp30_sm2": 122000.004000,
    "cintegrate_sp32_sm3": 121823.051337,
    "trainscan_p1": 122000.004030,        # includes sequential-sum rounding drift
    "trainscan_p1_exact": 122000.004000,  # what tree/look-back accumulation prints
    "trainscan_p7": 0.0,
    "trainscan_p16": 117642.707174,
    "train_analytic_1800": 121999.99983,
}
