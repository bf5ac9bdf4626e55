#!/usr/bin/env python3
"""One integration per call (the reference's timing unit: cintegrate.cu:102-104,127-141 and
riemann.cpp:49-51,90-93 clock exactly one run): launch -> pinned result, host-timed.

Forms, each the median of --reps calls after warmup, pi4 N = 1e9 fp64 on one GPU:
  direct      plan.run(): one fused (ticket) launch straight into pinned memory + stream sync
  graph1      a 1-step batch graph replay (+ its closing kernel) + stream sync
  native      RiemannPlan.time_one_shot (the C++ loop: no Python between launch and wait),
              every form it knows, when the extension has it
Prints one JSON line per form.
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = float(sys.argv[2]) if len(sys.argv) > 2 else 1e9
    from cuda_v_mpi_amd import Integrator, native

    m = native()
    integ = Integrator("pi4", n=int(n), slots=48)
    p = integ.plan
    out = []

    def timed(fn, label):
        for _ in range(200):  # warm + clocks
            fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e6)
        out.append({"form": label, "median_us": statistics.median(ts), "min_us": min(ts),
                    "max_us": max(ts), "reps": reps, "n": n, "grid": p.grid})

    timed(p.run, "direct_py")
    p.prepare_steps(1)
    timed(lambda: p.run_steps(1, False, True), "graph1_py")
    if hasattr(p, "time_one_shot"):
        for mode in ("direct", "graph", "direct_poll", "graph_poll"):
            try:
                r = p.time_one_shot(reps, mode, 400)
            except Exception as e:  # noqa: BLE001
                out.append({"form": "native_" + mode, "error": str(e)})
                continue
            r["form"] = "native_" + mode
            out.append(r)
    for r in out:
        print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
