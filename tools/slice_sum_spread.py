#!/usr/bin/env python3
"""How far may a G-GPU sum of rank slices sit from the 1-GPU value? Derived on ONE GPU.

A G-rank run (riemann --gpus G, miintrun -np G riemann, bench.py --gpus G) integrates each
rank's slice of [0, N) with that rank's own plan (its own auto grid, tile anchors starting
at its i_begin) and all-reduces the G scaled values; the 1-GPU run sums every tile in one
plan. Both are exact-grade fp64 sums of the same samples, but their roundings differ: the
slices move the series tiles' seeds and the lane/workgroup partials, and the all-reduce adds
the G values in an order RCCL picks (ring: a rotation; tree: pairs). This tool computes, on
one GPU, every rank's slice value exactly as that rank computes it
(RiemannConfig.slice_rank/slice_world: the same sample range, grid and kernels), sums them in
EVERY order an all-reduce may use — all G! left-to-right folds and the balanced pairwise tree
of every permutation — and records the spread against the 1-GPU value. The multi-GPU tests
(tests/test_multi_gpu.py) take their tolerance from this file: 4x the largest spread seen,
at least 4 ulp.

    python tools/slice_sum_spread.py [--out profiles/r6/slice_sum_spread.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EPS = 2.0 ** -52


def tree_sum(vals):
    vals = list(vals)
    while len(vals) > 1:
        nxt = [vals[i] + vals[i + 1] for i in range(0, len(vals) - 1, 2)]
        if len(vals) % 2:
            nxt.append(vals[-1])
        vals = nxt
    return vals[0]


def fold_sum(vals):
    s = 0.0
    for v in vals:
        s += v
    return s


def spread(vals, one):
    sums = set()
    for perm in itertools.permutations(vals):
        sums.add(fold_sum(perm))
        sums.add(tree_sum(perm))
    rel = [abs(s - one) / abs(one) for s in sums]
    return {"orders": len(sums), "max_rel": max(rel), "min_rel": min(rel),
            "sums": sorted(sums)[:4] + (["..."] if len(sums) > 8 else []) + sorted(sums)[-4:]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default="")
    ap.add_argument("--n", type=float, default=1e9)
    a = ap.parse_args(argv)
    from cuda_v_mpi_amd import Integrator

    n = int(a.n)
    rows = []
    tol = {}
    for integrand, rule in (("pi4", "mid"), ("pi4", "left"), ("sin", "mid")):
        one = Integrator(integrand, n=n, rule=rule).run().value
        for g in (2, 3, 4, 8):
            vals = []
            for r in range(g):
                it = Integrator(integrand, n=n, rule=rule, slice_of=(r, g))
                vals.append(it.run().value)
            sp = spread(vals, one)
            rows.append({"integrand": integrand, "rule": rule, "N": n, "G": g, "one_gpu": one,
                         "rank_values": vals, **sp, "max_ulps_of_value": sp["max_rel"] / EPS})
            key = f"{integrand}_{rule}_{g}"
            tol[key] = max(4 * sp["max_rel"], 4 * EPS)
            print(json.dumps(rows[-1]), flush=True)
    worst = {str(g): max(v for k, v in tol.items() if k.endswith(f"_{g}")) for g in (2, 3, 4, 8)}
    rec = {"what": "relative spread of G-slice sums vs the 1-GPU value over every all-reduce "
                   "order (fold and pairwise tree of every permutation); tolerance = 4x spread",
           "rows": rows, "tolerance_rel": tol, "tolerance_rel_by_g": worst}
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps({"tolerance_rel_by_g": worst}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
