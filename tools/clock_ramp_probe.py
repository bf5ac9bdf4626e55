#!/usr/bin/env python3
"""Time per step of the headline integration in consecutive chunks from a cold start.

    python tools/clock_ramp_probe.py [--chunks 40] [--chunk 50]

Shows how long the GPU takes to reach its steady per-step time after it starts working
(clock/power ramp), which decides how much warmup bench.py needs before its timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cuda_v_mpi_amd import Integrator  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=40)
    ap.add_argument("--chunk", type=int, default=48)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep before the run")
    a = ap.parse_args()
    plan = Integrator("pi4", n=10**9, backend="hip", slots=48).plan
    plan.launch_steps(48, False, True)  # capture + one batch
    plan.sync()
    if a.idle_ms:
        time.sleep(a.idle_ms / 1e3)
    rows, t_start = [], time.perf_counter()
    for c in range(a.chunks):
        t0 = time.perf_counter()
        plan.launch_steps(a.chunk, False, True)
        plan.sync()
        t1 = time.perf_counter()
        rows.append({"chunk": c, "t_ms": round((t0 - t_start) * 1e3, 2),
                     "us_per_step": round((t1 - t0) / a.chunk * 1e6, 2)})
    for r in rows:
        print(json.dumps(r), flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
