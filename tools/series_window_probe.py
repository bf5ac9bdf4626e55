#!/usr/bin/env python3
"""Per-point statistic of the `series` (g-fold) Pi4 division on the bench record's window
(64 K samples from index n/8 + 12345 at N = 1e9, left rule) against the IEEE path, in the
definition `tests/test_gpu_kernels.py::test_pi4_series_record_window` pins: max |d| in ulp of
the IEEE value, and the fractions of points with |d| <= 1 and <= 2. One JSON line.

    python tools/series_window_probe.py
"""
from __future__ import annotations

import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from cuda_v_mpi_amd.models import integrands
    from cuda_v_mpi_amd.ops import kernels

    n = 10**9
    spec = integrands.pi4()
    i0 = n // 8 + 12_345
    v = kernels.point_values(spec, n, rule="left", div="series", i_begin=i0, n_local=1 << 16)
    w = kernels.point_values(spec, n, rule="left", div="ieee", i_begin=i0, n_local=1 << 16)
    u = ((v - w) / (torch.nextafter(w.abs(), torch.full_like(w, math.inf)) - w.abs())).abs()
    print(json.dumps({"max": float(u.max()), "le1": float((u <= 1.0).double().mean()),
                      "le2": float((u <= 2.0).double().mean())}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
