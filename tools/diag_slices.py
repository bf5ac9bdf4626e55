#!/usr/bin/env python3
"""The diagnostic batch (RiemannPlan.diagnose_batch) at G = 1 and the per-GPU shares of a
G-GPU strong-scaled headline, next to a timed batch of the same plan, one JSON line each.

    python tools/diag_slices.py [--slices 1,2,4,8] [--steps 20] [--reps 5] [--collective]

Per share: the plan of rank 0's slice (slice_of=(0, G), N = 1e9 in total), 40 warm batches,
then `reps` times a timed batch (run_steps: wall and device span) followed by the diagnostic
batch (compute, close, all-reduce, copy, the event's own price, the host's part). With
--collective the plan runs its 1-rank RCCL stage, as a rank of a G-GPU job would
(profiles/r6/diag_slices.jsonl, batch_tail.md).
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
    ap.add_argument("--slices", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--collective", action="store_true")
    ap.add_argument("--close", default="auto")
    ap.add_argument("--with-comm", action="store_true",
                    help="create a 1-rank RCCL communicator first (its plans stay local): "
                         "does the communicator's presence change the batches?")
    a = ap.parse_args(argv)

    from cuda_v_mpi_amd import Integrator

    keep = None
    if a.with_comm:
        keep = Integrator("pi4", n=10**6, slots=a.steps, force_collective=True)
        keep.plan.run_steps(2, True, False)

    for g in (int(x) for x in a.slices.split(",")):
        it = Integrator("pi4", n=int(a.n), slots=a.steps, force_collective=a.collective,
                        slice_of=(0, g), close=a.close)
        for _ in range(40):
            it.plan.run_steps(a.steps, a.collective, False)
        for r in range(a.reps):
            t = it.plan.run_steps(a.steps, a.collective, False)
            d = it.plan.diagnose_batch(a.steps)
            print(json.dumps(dict(d, slice=g, rep=r, collective=a.collective,
                                  with_comm=keep is not None,
                                  close_in_launch=bool(it.plan.close_in_launch),
                                  host_us=d["wall_us"] - d["device_us"],
                                  timed_wall_us=t["wall_s"] * 1e6,
                                  timed_device_us=t["device_ms"] * 1e3)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
