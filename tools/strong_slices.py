#!/usr/bin/env python3
"""Per-GPU share of the fixed-N headline (N = 1e9 in total) for G = 1, 2, 4, 8, on ONE GPU.

The reference keeps N fixed and splits it over its workers (riemann.cpp:10,71-73). On an
8-GPU node each rank of `bench.py --gpus G` integrates 1/G of N = 1e9 and all-reduces its
partials over RCCL. This tool times exactly that per-GPU work on the one-GPU pool: rank 0's
slice (RiemannConfig.slice_rank/slice_world) in the same 48-step graph batches, with the
1-rank RCCL all-reduce stage captured in the graph (force_collective), so the slice table
shows the per-GPU latency floor a strong-scaled run would hit. Optional grid sweep.

    python tools/strong_slices.py [--gpus 1,2,4,8] [--grids 0,256,512,...] [--jsonl FILE]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(plan, steps: int, pipeline: bool, graphs: bool = True) -> float:
    """ms per step of graph-replayed (or directly launched) batches, after >= 30 ms of the
    same batches."""
    plan.prepare_steps(steps)
    t = time.perf_counter()
    plan.launch_steps(steps, pipeline, graphs)
    plan.sync()
    reps = max(1, math.ceil(0.03 / max(time.perf_counter() - t, 1e-6)))
    for _ in range(reps):
        plan.launch_steps(steps, pipeline, graphs)
    plan.sync()
    best = math.inf
    for _ in range(5):
        t = time.perf_counter()
        plan.launch_steps(steps, pipeline, graphs)
        plan.sync()
        best = min(best, (time.perf_counter() - t) / steps * 1e3)
    return best


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--collective", choices=["on", "off", "both"], default="both")
    ap.add_argument("--step-streams", default="0", help="comma list (0 = the plan's auto)")
    ap.add_argument("--graphs", choices=["on", "off", "both"], default="on",
                    help="batches as graph replays, direct launches, or both")
    ap.add_argument("--close", default="auto",
                    help="comma list of multi-step batch closes: auto, kernel, launch")
    ap.add_argument("--ar-host", default="on", choices=["on", "off", "both"],
                    help="bucketed all-reduce straight into pinned memory (on), or in place "
                         "on the device + a copy (off)")
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)

    from cuda_v_mpi_amd import Integrator

    n = int(a.n)
    rows = []
    modes = {"on": [True], "off": [False], "both": [True, False]}[a.collective]
    gmodes = {"on": [True], "off": [False], "both": [True, False]}[a.graphs]
    armodes = {"on": [True], "off": [False], "both": [True, False]}[a.ar_host]
    configs = [(gr, c, q, gm, cl, ar) for gr in (int(x) for x in a.grids.split(","))
               for c in modes for q in (int(y) for y in a.step_streams.split(","))
               for gm in gmodes for cl in a.close.split(",") for ar in armodes]
    for g in (int(x) for x in a.gpus.split(",")):
        for grid, coll, ss, gm, cl, ar in configs:
            it = Integrator("pi4", n=n, slots=48, grid=grid, force_collective=coll,
                            slice_of=(0, g), step_streams=ss, close=cl, allreduce_to_host=ar)
            ms = timed(it.plan, a.steps, coll, gm)
            v = it.plan.host_result(it.plan.host_index_of(a.steps - 1, True))
            # rank 0's slice of [0, 1): its exact integral is 4 atan(x1)
            x1 = it.plan.count / n
            err = abs(v - 4.0 * math.atan(x1))
            row = {"G": g, "n_total": n, "n_per_gpu": it.plan.count,
                   "grid": it.plan.grid, "grid_arg": grid, "rccl_stage": coll,
                   "step_streams": it.plan.step_streams(a.steps), "graphs": gm,
                   "close": cl, "close_in_launch": it.plan.close_in_launch,
                   "allreduce_to_host": it.plan.allreduce_to_host,
                   "result": v,
                   "ms_per_step": ms, "us_per_step": ms * 1e3,
                   "per_gpu_subint_per_s": it.plan.count / (ms * 1e-3),
                   "projected_strong_value": n / (ms * 1e-3),
                   "slice_abs_err": err, "steps": a.steps}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del it
    key = lambda r: (r["grid_arg"], r["rccl_stage"], r["step_streams"], r["graphs"],  # noqa: E731
                     r["close"], r["allreduce_to_host"])
    base = {key(r): r["ms_per_step"] for r in rows if r["G"] == 1}
    for r in rows:
        b = base.get(key(r))
        if b:
            r["projected_strong_eff"] = b / (r["G"] * r["ms_per_step"])
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
