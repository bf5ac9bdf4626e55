#!/usr/bin/env python3
"""fp32 accumulation policy (BASELINE #4: "packed-fp32 wave reduction; error vs fp64").

Times the same 4/(1+x^2) integral three ways on one GPU — fp64; fp32 samples with the tile
values folded into fp64 lane sums (dtype fp32, the default fp32 path); fp32 samples with
fp32 lane sums, v_add_f32_dpp wave reduction and an fp32 block step (dtype fp32acc) — and
reports each one's error against pi and against the fp64 value.

    python tools/fp32_accum.py [--n 1e9,1e8] [--rule left,mid] [--jsonl FILE]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(plan, steps=48):
    plan.prepare_steps(steps)
    t = time.perf_counter()
    plan.launch_steps(steps, False, True)
    plan.sync()
    for _ in range(max(1, math.ceil(0.05 / max(time.perf_counter() - t, 1e-6)))):
        plan.launch_steps(steps, False, True)
    plan.sync()
    best = math.inf
    for _ in range(5):
        t = time.perf_counter()
        plan.launch_steps(steps, False, True)
        plan.sync()
        best = min(best, (time.perf_counter() - t) / steps * 1e3)
    return best, plan.host_result(plan.host_index_of(steps - 1, True))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1e9,1e8")
    ap.add_argument("--rule", default="left,mid")
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)
    from cuda_v_mpi_amd import Integrator

    rows = []
    for n in (int(float(x)) for x in a.n.split(",")):
        for rule in a.rule.split(","):
            ref = None
            for dt in ("fp64", "fp32", "fp32acc"):
                it = Integrator("pi4", n=n, rule=rule, dtype=dt, slots=48)
                ms, v = timed(it.plan)
                ref = v if dt == "fp64" else ref
                row = {"n": n, "rule": rule, "dtype": dt,
                       "accum": {"fp64": "fp64", "fp32": "fp64-fold", "fp32acc": "fp32"}[dt],
                       "ms_per_step": ms, "subint_per_s": n / (ms * 1e-3), "result": v,
                       "abs_err": abs(v - math.pi), "rel_diff_vs_fp64": abs(v - ref) / ref}
                rows.append(row)
                print(json.dumps(row), flush=True)
                del it
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
