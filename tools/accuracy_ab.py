#!/usr/bin/env python3
"""Per-point accuracy against speed for pi4 N = 1e9 fp64.

For each division mode — series (the headline: g = 1/2 + e, one square per sample),
series_exact (the residuals kept at their own precision: e + e^2 per sample) and ieee
(correctly rounded division per sample) — one line with:
  * us per integration: 48-step graph batches (multi-step launches where they pay), best of
    5 timed batches after ~50 ms of settle replays;
  * the ulp histogram of every sample's value against IEEE division, over 4 windows of 64 K
    samples spread across [0, 1] (x ~ 0.01, 0.3, 0.6, 0.95);
  * every sample's error against the true value at the true coordinate, 4 / (1 + (i h)^2) in
    x87 extended precision (64-bit significand; numpy longdouble), in ulps of the fp64 result:
    IEEE division per sample is not exact either — it rounds the coordinate fma(u, h, x0),
    then 1 + x^2, then the quotient — so "ulp vs IEEE" mixes the two paths' errors.

    python tools/accuracy_ab.py > gpurun_out/accuracy_ab.jsonl
"""
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    import numpy as np
    import torch

    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.ops import kernels

    n = 10**9
    steps = 48
    spec = Integrator("pi4", n=n, backend="cpu").spec
    # the window at x = 0 (values just under 4: where 1 + x^2 rounds least, round 4's worst
    # for series_exact) and four spread across [0, 1]
    windows = [0] + [int(f * n) + 12_345 for f in (0.01, 0.3, 0.6, 0.95)]
    w = 1 << 16
    ref = {i0: kernels.point_values(spec, n, rule="left", div="ieee", i_begin=i0, n_local=w)
           for i0 in windows}
    h = np.longdouble(float(1.0 / n))  # the kernels' h: fp64 (b - a) / n
    truth = {}
    for i0 in windows:
        x = (np.arange(w, dtype=np.longdouble) + np.longdouble(i0)) * h
        truth[i0] = np.longdouble(4) / (np.longdouble(1) + x * x)
    for div in ("series", "series_exact", "ieee"):
        it = Integrator("pi4", n=n, div=div, slots=steps)
        p = it.plan
        p.prepare_steps(steps)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.05:
            p.launch_steps(steps, False, True)
        p.sync()
        best = min(p.run_steps(steps, False, True)["device_ms"] for _ in range(5)) / steps
        v = p.host_result(p.host_index_of(steps - 1, True))
        hist = {"<=0.5": 0, "<=1": 0, "<=2": 0, "<=3": 0, "<=5": 0, ">5": 0}
        umax, total = 0.0, 0
        tmax, tsum, t1 = 0.0, 0.0, 0
        per_window = []
        for i0 in windows:
            val = kernels.point_values(spec, n, rule="left", div=div, i_begin=i0, n_local=w)
            tv = truth[i0]
            ut = np.abs((val.cpu().numpy().astype(np.longdouble) - tv) /
                        np.spacing(tv.astype(np.float64)).astype(np.longdouble)).astype(np.float64)
            tmax = max(tmax, float(ut.max()))
            tsum += float(ut.sum())
            per_window.append({"i0": i0, "x0": i0 / n, "vs_true_max_ulp": float(ut.max()),
                               "vs_true_mean_ulp": float(ut.mean())})
            t1 += int((ut <= 1.0).sum())
            r = ref[i0]
            spacing = torch.nextafter(r.abs(), torch.full_like(r, math.inf)) - r.abs()
            u = ((val - r) / spacing).abs().cpu()
            umax = max(umax, float(u.max()))
            total += u.numel()
            prev = torch.zeros_like(u, dtype=torch.bool)
            for k, lim in (("<=0.5", 0.5), ("<=1", 1.0), ("<=2", 2.0), ("<=3", 3.0), ("<=5", 5.0)):
                m = u <= lim
                hist[k] += int((m & ~prev).sum())
                prev = m
            hist[">5"] += int((~prev).sum())
        cum1 = (hist["<=0.5"] + hist["<=1"]) / total
        cum2 = cum1 + hist["<=2"] / total
        print(json.dumps({
            "div": div, "effective_div": str(p.effective_div).split(".")[-1],
            "multistep": bool(p.multistep), "grid": p.grid, "us_per_integration": best * 1e3,
            "subint_per_s": n / (best * 1e-3), "result": v, "abs_err": abs(v - math.pi),
            "points": total, "max_ulp": umax, "frac_within_1ulp": cum1,
            "frac_within_2ulp": cum2, "ulp_hist": hist,
            "vs_true_max_ulp": tmax, "vs_true_mean_ulp": tsum / total,
            "vs_true_frac_within_1ulp": t1 / total, "windows": per_window}), flush=True)
        del it, p
    return 0


if __name__ == "__main__":
    sys.exit(main())
