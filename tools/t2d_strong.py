#!/usr/bin/env python3
"""Per-GPU share of the 2-D field (BASELINE #5, 4096^2) for G = 1, 2, 4, 8, on ONE GPU.

On an 8-GPU node `bench.py --gpus G` splits the field's sample rows over G ranks; each rank
replays its row slice in multi-step graph batches and closes every replay with ONE RCCL
all-reduce of the replay's per-integration partials (Table2DPlan, bucketed). This tool times
exactly that per-GPU work on the one-GPU pool: rank 0's row slice (Table2DConfig rank/world)
with a 1-rank RCCL communicator and the all-reduce + copy stage captured in each replay
(force_collective), and projects the fixed-work efficiency t(1) / (G t(G)) — what
`scaling.py` reports as `t2d_strong_eff` from a real G-GPU run, minus the cross-GPU hops.

    python tools/t2d_strong.py [--gpus 1,2,4,8] [--grid 4096] [--collective on|off|both]
        [--graph-steps 0] [--reps 3] [--jsonl FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--collective", choices=["on", "off", "both"], default="both")
    ap.add_argument("--graph-steps", type=int, default=0, help="per replay (0 = the plan's auto)")
    ap.add_argument("--reps", type=int, default=3, help="timed calls per point (best kept)")
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)

    from cuda_v_mpi_amd import native
    from cuda_v_mpi_amd.parallel.dist import DistContext, native_comm

    m = native()
    ctx = DistContext(rank=0, world=1, local_rank=0, device=0)
    comm = native_comm(ctx)  # 1 rank: the RCCL stage's kernels, no cross-GPU hop
    modes = {"on": [True], "off": [False], "both": [True, False]}[a.collective]
    rows = []
    for g in (int(x) for x in a.gpus.split(",")):
        for coll in modes:
            p = m.Table2DPlan(a.grid, 1800.0, 0, comm if coll else None, True, True, 0, 0, g,
                              graph_steps=a.graph_steps, force_collective=coll)
            assert p.collective == coll and p.bucketed == coll
            p.run()
            ms = min(p.time(p.graph_steps * 4, True) for _ in range(a.reps))
            row = {"G": g, "grid": a.grid, "rows": [p.row0, p.row1], "rccl_stage": coll,
                   "graph_steps": p.graph_steps, "phases": p.phases, "workgroups": p.workgroups,
                   "us_per_integration": ms * 1e3, "partial": p.last_result()}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del p
    base = {r["rccl_stage"]: r["us_per_integration"] for r in rows if r["G"] == 1}
    for r in rows:
        b = base.get(r["rccl_stage"])
        if b:
            r["projected_t2d_strong_eff"] = b / (r["G"] * r["us_per_integration"])
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    for r in rows:
        print(f"G={r['G']} rccl_stage={r['rccl_stage']} {r['us_per_integration']:.3f} us "
              f"eff={r.get('projected_t2d_strong_eff', float('nan')):.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
