#!/usr/bin/env python3
"""Host-side cost of bench.py's timed region on one GPU: how long the driver-shape K-step
region takes on the host clock against the device time of the same replay (hipEvents), for
several ways of waiting for the replay.

    python tools/host_sync_probe.py [--steps 20] [--reps 30] [--jsonl FILE]

Forms (each: launch_steps(K) on the plan's compute stream, then ...):
  plan_sync    plan.sync() (hipStreamSynchronize) + torch.cuda.synchronize()   (bench.py today)
  poll         native.wait_with_timeout(compute stream) (hipStreamQuery spin) + torch sync
  torch_only   torch.cuda.synchronize() alone
  direct_plan_sync   the batch's two kernels launched directly (no graph), plan.sync + torch
The device span comes from hipEvents recorded around the same launch (separate reps).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)

    import torch

    from cuda_v_mpi_amd import Integrator, native

    m = native()
    it = Integrator("pi4", n=10**9, rule="left", slots=max(48, a.steps))
    plan = it.plan
    K = a.steps
    plan.prepare_steps(K)
    cs = plan.compute_stream
    stream = torch.cuda.ExternalStream(cs)

    def settle(ms=60.0):
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < ms:
            plan.launch_steps(K, True, True)
            plan.sync()

    def idle_sync():
        torch.cuda.synchronize()

    forms = {
        "plan_sync": (True, lambda: (plan.sync(), torch.cuda.synchronize())),
        "poll": (True, lambda: (m.wait_with_timeout(cs, 60.0), torch.cuda.synchronize())),
        "torch_only": (True, lambda: torch.cuda.synchronize()),
        # the batch's two kernels launched directly instead of as a graph replay
        "direct_plan_sync": (False, lambda: (plan.sync(), torch.cuda.synchronize())),
    }
    rows = []
    settle()
    for rep in range(a.reps):
        for name, (graphs, wait) in forms.items():
            idle_sync()
            t0 = time.perf_counter()
            plan.launch_steps(K, True, graphs)
            wait()
            rows.append((name, (time.perf_counter() - t0) * 1e6))
        for graphs in (True, False):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            idle_sync()
            e0.record(stream)
            plan.launch_steps(K, True, graphs)
            e1.record(stream)
            torch.cuda.synchronize()
            rows.append(("device_events" if graphs else "direct_device_events",
                         e0.elapsed_time(e1) * 1e3))
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        rows.append(("idle_torch_sync", (time.perf_counter() - t0) * 1e6))
        t0 = time.perf_counter()
        plan.sync()
        rows.append(("idle_plan_sync", (time.perf_counter() - t0) * 1e6))
    out = {}
    for name in dict.fromkeys(r[0] for r in rows):
        v = [r[1] for r in rows if r[0] == name]
        out[name] = {"median_us": statistics.median(v), "min_us": min(v), "max_us": max(v)}
    rec = {"steps": K, "reps": a.reps, "forms": out,
           "median_us_per_step": {k: v["median_us"] / K for k, v in out.items()
                                  if not k.startswith("idle")}}
    print(json.dumps(rec, indent=1))
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
