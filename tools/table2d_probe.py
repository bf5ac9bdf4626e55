#!/usr/bin/env python3
"""Time the 2-D field kernel (BASELINE #5) per launch: the whole grid and one GPU's row slice
of an 8-GPU split, at 4096^2 and 8192^2 (torch events around 200 back-to-back launches).

    python tools/table2d_probe.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cuda_v_mpi_amd.ops import kernels  # noqa: E402
from cuda_v_mpi_amd.utils import fixtures  # noqa: E402


def timed(fn, iters: int = 200) -> float:
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main() -> None:
    v = torch.as_tensor(fixtures.profile_table(), device="cuda")
    T = kernels.outer_product(v)
    for g in (4096, 8192):
        full = timed(lambda: kernels.table2d(T, 1800.0, 1800.0, g, g))
        s = g // 8
        part = timed(lambda: kernels.table2d(T, 1800.0, 1800.0, g, g, 3 * s, 4 * s))
        print(json.dumps({"grid": g, "full_us": round(full, 2), "eighth_rows_us": round(part, 2),
                          "samples_per_s_full": g * g / full * 1e6}), flush=True)


if __name__ == "__main__":
    main()
