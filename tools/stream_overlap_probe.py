#!/usr/bin/env python3
"""Probe: do independent integrations on several streams overlap one kernel's ramp/tail with
the next one's work? (Per-kernel fixed cost is ~2-3 us: at 1/8 of N = 1e9 a step takes
11.5 us against 8.4 us of VALU work, profiles/r3/strong_slices.jsonl.)

Each step is a complete fused integration (own write-once partial slots and ticket, own
result). Steps are dealt round-robin to S streams; direct launches and a torch.cuda graph
capture of the same fork/join pattern are timed.

    python tools/stream_overlap_probe.py [--n 1.25e8] [--streams 1,2,3,4] [--grids 512]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1.25e8)
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--grids", default="512")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)

    import torch

    from cuda_v_mpi_amd.models import integrands
    from cuda_v_mpi_amd.ops import kernels

    spec = integrands.pi4()
    n = int(a.n)
    rows = []
    for grid in (int(g) for g in a.grids.split(",")):
        for S in (int(s) for s in a.streams.split(",")):
            streams = [torch.cuda.Stream() for _ in range(S)]
            ws = [kernels.FusedWorkspace(grid) for _ in range(S)]
            out = torch.zeros(a.steps, dtype=torch.float64, device="cuda")

            def body():
                main = torch.cuda.current_stream()
                ev = torch.cuda.Event()
                ev.record(main)
                for s in streams:
                    s.wait_event(ev)
                for k in range(a.steps):
                    with torch.cuda.stream(streams[k % S]):
                        kernels.riemann(spec, n, rule="left", grid=grid, workspace=ws[k % S],
                                        out=out[k:k + 1])
                for s in streams:
                    e = torch.cuda.Event()
                    e.record(s)
                    main.wait_event(e)

            def timed(fn, reps=20):
                fn()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(max(1, math.ceil(0.03 / max(1e-6, 1e-5 * a.steps)))):
                    fn()
                torch.cuda.synchronize()
                best = math.inf
                for _ in range(reps):
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    fn()
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t) / a.steps * 1e6)
                return best

            direct_us = timed(body)
            side = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                body()  # warm outside capture
            torch.cuda.synchronize()
            graph_us = None
            try:
                with torch.cuda.graph(g, stream=side):
                    body()
                graph_us = timed(g.replay)
            except Exception as e:  # noqa: BLE001
                graph_us = f"{type(e).__name__}: {e}"
            vals = out.tolist()
            err = max(abs(v - math.pi - 1.0 / n) for v in vals)
            row = {"n": n, "grid": grid, "streams": S, "direct_us_per_step": direct_us,
                   "graph_us_per_step": graph_us, "max_err_minus_h": err}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
