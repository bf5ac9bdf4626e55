#!/usr/bin/env python3
"""Per-point error of the angle-addition series (sin / train velocity) and of the per-sample
ocml path, both against an x87 long-double evaluation of the same samples on the host.

    python tools/series_exact_probe.py [--n 1e9] [--windows 16] [--width 65536]

The two device paths round differently: the series takes every sample's angle exactly from
the tile midpoint (host long-double cos/sin(k delta)); the per-sample path rounds each
coordinate x0 + u h and then t / ts. Comparing each with a long-double reference separates
the two (tests/test_gpu_kernels.py only bounds their difference).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cuda_v_mpi_amd.models import integrands  # noqa: E402
from cuda_v_mpi_amd.ops import kernels  # noqa: E402


def exact(spec, n: int, i0: int, m: int) -> np.ndarray:
    ld = np.longdouble
    i = np.arange(i0, i0 + m, dtype=np.float64).astype(ld)
    h = (ld(spec.b) - ld(spec.a)) / ld(n)
    x = ld(spec.a) + i * h  # left rule
    if spec.name == "sin":
        return np.sin(x)
    if spec.name == "train":
        return (ld(1) - np.cos(x / ld(spec.p0))) * ld(spec.p1)
    raise ValueError(spec.name)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--windows", type=int, default=16)
    ap.add_argument("--width", type=int, default=1 << 16)
    a = ap.parse_args()
    n = int(a.n)
    for spec in (integrands.sin(), integrands.train()):
        scale = 1.0 if spec.name == "sin" else spec.p1
        worst = {"series": 0.0, "ieee": 0.0}
        for w in range(a.windows):
            i0 = (n - a.width) * w // max(1, a.windows - 1)
            ref = exact(spec, n, i0, a.width)
            for div in worst:
                v = kernels.point_values(spec, n, rule="left", div=div, i_begin=i0, n_local=a.width)
                d = np.abs(v.cpu().numpy().astype(np.longdouble) - ref).max()
                worst[div] = max(worst[div], float(d))
        ulp = 2.0 ** -52 * scale
        print(f"{spec.name} n={n}: max |err| series {worst['series']:.3e} ({worst['series'] / ulp:.2f} ulp(scale)), "
              f"per-sample ocml {worst['ieee']:.3e} ({worst['ieee'] / ulp:.2f} ulp(scale))", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
