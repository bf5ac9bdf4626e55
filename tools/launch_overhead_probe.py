#!/usr/bin/env python3
"""Where the host-timed step exceeds the device span: launch call, stream sync, torch sync.

bench.py times K steps as barrier + sync | launch_steps(K) + plan.sync() + torch sync | on
the host. For K = 20 the device span is ~20 x 72.4 us, the host clock ~50 us more. This
probe splits that overhead for one host wait policy (argv[1]: none|auto|spin|yield|blocking,
set before the plan is built) and prints one JSON line.

    python tools/launch_overhead_probe.py spin
    python tools/launch_overhead_probe.py none 20 0      # third arg 0: direct enqueue, no graph
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    mode = sys.argv[1] if len(sys.argv) > 1 else "none"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    graphs = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
    from cuda_v_mpi_amd import native

    m = native()
    if mode != "none":
        m.set_device_flags(mode)
    import torch

    from cuda_v_mpi_amd import Integrator

    p = Integrator("pi4", n=10**9, slots=48).plan
    if graphs:
        p.prepare_steps(steps)
    for _ in range(60):  # warm + clock settle
        p.launch_steps(steps, False, graphs)
    p.sync()
    launch, psync, tsync, total = [], [], [], []
    for _ in range(40):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.launch_steps(steps, False, graphs)
        t1 = time.perf_counter()
        p.sync()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        launch.append(t1 - t0)
        psync.append(t2 - t1)
        tsync.append(t3 - t2)
        total.append(t3 - t0)
    dev = [p.run_steps(steps, False, graphs)["device_ms"] for _ in range(20)]
    med = lambda v: statistics.median(v) * 1e6  # noqa: E731
    rec = {"mode": mode, "flags": m.get_device_flags(), "steps": steps, "graphs": graphs,
           "multistep": bool(p.multistep),
           "launch_us": med(launch), "plan_sync_us": med(psync), "torch_sync_us": med(tsync),
           "host_total_us": med(total), "host_min_us": min(total) * 1e6,
           "device_event_us": statistics.median(dev) * 1e3,
           "host_us_per_step": med(total) / steps}
    rec["overhead_us"] = rec["host_total_us"] - rec["device_event_us"]
    print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
