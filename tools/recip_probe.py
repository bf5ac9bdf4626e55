#!/usr/bin/env python3
"""Bitwise check of the kIeee Pi4 reciprocal (integrands.hpp Pi4::recip_narrow) against IEEE
division over many random divisors on the GPU.

    python tools/recip_probe.py --batches 64 --out gpurun_out/recip_probe.json

Each batch draws 2^26 divisors (half uniform in [1, 2), half with random significands at
random exponents 0..499) and compares the kernel's reciprocal with torch's 1.0 / d on the
same device (the compiler's full IEEE division) bit for bit. Prints and writes one JSON
record: operands checked, mismatches, the first few mismatching divisors.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cuda_v_mpi_amd.ops import kernels  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=64)
    ap.add_argument("--log2-batch", type=int, default=26)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(a.seed)
    m = 1 << a.log2_batch
    checked, bad, first = 0, 0, []
    t0 = time.time()
    for b in range(a.batches):
        half = m // 2
        uni = 1.0 + torch.rand(half, generator=g, dtype=torch.float64, device=dev)
        exps = torch.randint(0, 500, (m - half,), generator=g, device=dev)
        wide = torch.ldexp(1.0 + torch.rand(m - half, generator=g, dtype=torch.float64,
                                            device=dev), exps)
        d = torch.cat([uni, wide])
        got = kernels.pi4_recip_narrow(d)
        want = 1.0 / d
        diff = got.view(torch.int64) != want.view(torch.int64)
        nb = int(diff.sum())
        if nb and len(first) < 8:
            first += d[diff][: 8 - len(first)].tolist()
        bad += nb
        checked += m
        if b % 16 == 15:
            print(f"batch {b + 1}/{a.batches}: {checked:.3e} checked, {bad} mismatches "
                  f"({time.time() - t0:.1f} s)", flush=True)
    rec = {"probe": "pi4_recip_narrow vs IEEE 1/d (torch on the same GPU)", "checked": checked,
           "mismatches": bad, "first_mismatching_d": first, "seed": a.seed,
           "device": torch.cuda.get_device_name(dev), "seconds": time.time() - t0}
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(rec) + "\n")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
