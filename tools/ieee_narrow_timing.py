#!/usr/bin/env python3
"""Time the kIeee Pi4 paths (fp64 and fp32) with the narrow-range reciprocal and with the
full library division (set_pi4_library_division) at the same N, and check the sums are
bitwise equal. One JSON line per (dtype, division).

    python tools/ieee_narrow_timing.py [--n 1e9] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cuda_v_mpi_amd import native  # noqa: E402
from cuda_v_mpi_amd.models import integrands  # noqa: E402
from cuda_v_mpi_amd.ops import kernels  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = int(a.n)
    m = native()
    spec = integrands.pi4()
    ws = kernels.FusedWorkspace(kernels.default_grid())
    out = torch.empty(1, dtype=torch.float64, device="cuda")
    vals = {}
    for dtype in ("fp64", "fp32"):
        for lib in (False, True):
            m.set_pi4_library_division(lib)
            try:
                run = lambda: kernels.riemann(spec, n, dtype=dtype, div="ieee", out=out,  # noqa: E731
                                              workspace=ws)
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                v = float(out.item())
            finally:
                m.set_pi4_library_division(False)
            vals[(dtype, lib)] = v
            print(json.dumps({"dtype": dtype, "division": "library" if lib else "narrow",
                              "N": n, "ms": ms, "subint_per_s": n / (ms * 1e-3), "result": v,
                              "bitwise_equal_to_narrow": None if not lib else
                              v == vals[(dtype, False)]}), flush=True)
    return 0 if all(vals[(d, True)] == vals[(d, False)] for d in ("fp64", "fp32")) else 1


if __name__ == "__main__":
    raise SystemExit(main())
