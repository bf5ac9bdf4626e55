#!/usr/bin/env python3
"""Fixed cost of one timed batch of the headline (pi4 N = 1e9 fp64, one GPU), as bench.py
times it (device sync, launch of K steps, plan sync, device sync; wall clock), for K = 1..48,
through a captured graph and through direct launches (the same multi-step kernel + close
kernel, enqueued without a graph). A fit T(K) = a K + b splits the per-step time a from the
per-batch cost b (launch, ramp, tail, close kernel, the syncs). One JSON line per (mode, K).

    python tools/replay_overhead_probe.py > gpurun_out/replay_overhead.jsonl
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    import torch

    from cuda_v_mpi_amd import Integrator

    it = Integrator("pi4", n=10**9, slots=48)
    p = it.plan
    ks = (1, 2, 5, 10, 20, 48)
    for k in ks:
        p.prepare_steps(k)
    # settle the clocks: ~60 ms of 20-step batches
    t = time.perf_counter()
    while time.perf_counter() - t < 0.06:
        p.launch_steps(20, False, True)
    p.sync()
    fits = {}
    for graphs in (True, False):
        pts = []
        for k in ks:
            walls = []
            for _ in range(7):
                for _ in range(3):  # keep the clocks up between timed batches
                    p.launch_steps(20, False, True)
                p.sync()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                p.launch_steps(k, False, graphs)
                p.sync()
                torch.cuda.synchronize()
                walls.append((time.perf_counter() - t0) * 1e6)
            w = statistics.median(walls)
            dev = p.run_steps(k, False, graphs)["device_ms"] * 1e3
            pts.append((k, w))
            print(json.dumps({"graphs": graphs, "steps": k, "wall_us": w, "wall_min_us": min(walls),
                              "device_us": dev, "us_per_step": w / k}), flush=True)
        n = len(pts)
        mx = sum(k for k, _ in pts) / n
        my = sum(w for _, w in pts) / n
        a = sum((k - mx) * (w - my) for k, w in pts) / sum((k - mx) ** 2 for k, _ in pts)
        fits["graph" if graphs else "direct"] = {"a_us_per_step": a, "b_us_per_batch": my - a * mx}
    print(json.dumps({"fit": fits}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
