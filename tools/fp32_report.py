#!/usr/bin/env python3
"""fp32 vs fp64 for every integrand (BASELINE #4 "fp32 path ... error vs fp64").

    python tools/fp32_report.py > profiles/r2/fp32_errors.jsonl

Per integrand, division mode and N in {1e3, 1e6, 1e9}: the packed-fp32 result, the fp64
result of the same kernel family, the fp64 torch reference where affordable (N <= 1e6) and
the relative differences.
"""
from __future__ import annotations

import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_v_mpi_amd.models import integrands  # noqa: E402
from cuda_v_mpi_amd.ops import kernels  # noqa: E402


def ref_sum(spec, n):
    h = (spec.b - spec.a) / n
    parts = []
    for s in range(0, n, 1 << 22):
        i = torch.arange(s, min(n, s + (1 << 22)), dtype=torch.float64, device="cuda")
        parts.append(float(spec.f_torch(spec.a + (i + 0.5) * h).sum()))
    return math.fsum(parts) * h


def main() -> int:
    specs = [integrands.pi4(), integrands.sin(), integrands.train(), integrands.table(),
             integrands.poly(seed=3)]
    for spec in specs:
        for n in (10**3, 10**6, 10**9):
            for div in ("series", "ieee"):
                f32 = float(kernels.riemann(spec, n, rule="mid", dtype="fp32", div=div).item())
                f64 = float(kernels.riemann(spec, n, rule="mid", dtype="fp64", div=div).item())
                ref = ref_sum(spec, n) if n <= 10**6 else None
                rec = dict(integrand=spec.name, n=n, div=div, rule="mid", fp32=f32, fp64=f64,
                           rel_fp32_vs_fp64=abs(f32 - f64) / abs(f64),
                           torch_fp64=ref,
                           rel_fp32_vs_torch=None if ref is None else abs(f32 - ref) / abs(ref),
                           analytic=spec.analytic(),
                           abs_err_fp32=abs(f32 - spec.analytic()),
                           abs_err_fp64=abs(f64 - spec.analytic()))
                print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
