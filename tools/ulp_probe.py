#!/usr/bin/env python3
"""Per-point error of the Pi4 series path vs IEEE division, in units of ulp(IEEE value),
over the whole domain at several step sizes: max, histogram of round(|d|) (so the "1 ulp" bin
holds |d| < 1.5) and the exact fractions with |d| <= 1 and |d| <= 2."""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cuda_v_mpi_amd.models import integrands  # noqa: E402
from cuda_v_mpi_amd.ops import kernels  # noqa: E402

spec = integrands.pi4()
CH = 1 << 20
for n in (10**9, 10**8, 33_000_000):
    hist = torch.zeros(8, dtype=torch.int64)
    le1 = le2 = 0
    worst = 0.0
    ssum, cnt = 0.0, 0
    for i0 in range(0, n - CH, (n - CH) // 32):
        v = kernels.point_values(spec, n, rule="left", div="series", i_begin=i0, n_local=CH)
        w = kernels.point_values(spec, n, rule="left", div="ieee", i_begin=i0, n_local=CH)
        sp = torch.nextafter(w.abs(), torch.full_like(w, math.inf)) - w.abs()
        su = (v - w) / sp
        ssum += float(su.sum())
        cnt += su.numel()
        u = su.abs()
        le1 += int((u <= 1.0).sum())
        le2 += int((u <= 2.0).sum())
        worst = max(worst, float(u.max()))
        hist += torch.bincount(torch.clamp(u.round().long(), max=7).cpu(), minlength=8)
    tot = int(hist.sum())
    print(f"n={n:.3g}: max {worst:.3f} ulp; signed mean {ssum / cnt:+.4f} ulp; distribution (0,1,2,3+ ulp): "
          + ", ".join(f"{int(hist[k])/tot:.4f}" for k in range(3)) + f", {int(hist[3:].sum())/tot:.2e}"
          + f"; |d| <= 1: {le1 / cnt:.4f}, |d| <= 2: {le2 / cnt:.4f}")
