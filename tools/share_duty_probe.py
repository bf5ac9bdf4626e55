#!/usr/bin/env python3
"""Does a share's batch cost depend on how busy the GPU was just before it?

    python tools/share_duty_probe.py [--slices 1,4,8] [--steps 20] [--reps 30]

Per share of N = 1e9 (slice_of=(0, G), one GPU, no collective), three ways of running the
same 20-step batch, in rotating order:

  back_to_back  K batches enqueued without a host sync between them, then one sync: the
                GPU never idles (miint bench's loop, bench.py's settle phase);
  synced        one batch per host round trip (RiemannPlan.run_steps: sync, launch, sync):
                the GPU idles for the host's turnaround between batches (tools/diag_slices.py,
                strong_slices.py, batch_ab.py);
  driver        bench.py's timed region: ~60 ms of back-to-back batches, a sync, then ONE
                batch timed from its launch call to its sync;
  after_settle_3rd, short_settle, idle_1ms, second, devsync, warm1
                the same with the third / second batch after the settle, a 5-batch settle,
                1 ms of idle GPU, a device-wide sync or a 1-step batch before the batch:
                which part of `driver` costs;
  bench_like    bench.py's timed region after its re-arm batch, with the launch call, the
                plan's sync and torch.cuda.synchronize() timed apart.

Host microseconds per batch (median over reps) for each. profiles/r6/batch_tail.md.
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
    ap.add_argument("--slices", default="1,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--batches", type=int, default=50, help="K of back_to_back")
    ap.add_argument("--settle-ms", type=float, default=60.0)
    ap.add_argument("--idle-us", default="",
                    help="instead: the re-arm batch, then this many us of idle GPU (a list), "
                         "then the batch")
    a = ap.parse_args(argv)

    import torch

    from cuda_v_mpi_amd import Integrator

    for g in (int(x) for x in a.slices.split(",")):
        it = Integrator("pi4", n=10**9, slots=a.steps, slice_of=(0, g))
        p, S = it.plan, a.steps
        for _ in range(20):
            p.run_steps(S, False, False)
        t = time.perf_counter()
        p.launch_steps(S, False, False)
        p.sync()
        per = max(time.perf_counter() - t, 1e-6)
        settle = max(1, int(a.settle_ms * 1e-3 / per))
        res = {"back_to_back": [], "synced": [], "driver": []}

        def back_to_back():
            p.sync()
            t0 = time.perf_counter()
            for _ in range(a.batches):
                p.launch_steps(S, False, False)
            p.sync()
            return (time.perf_counter() - t0) / a.batches

        def synced():
            return p.run_steps(S, False, False)["wall_s"]

        launch_call = {"driver": [], "after_settle_3rd": [], "short_settle": [], "second": [],
                       "devsync": [], "warm1": []}

        def one(tag):  # one batch from its launch call to its sync; the call's own share
            t0 = time.perf_counter()
            p.launch_steps(S, False, False)
            t1 = time.perf_counter()
            p.sync()
            t2 = time.perf_counter()
            if tag:
                launch_call[tag].append((t1 - t0) * 1e6)
            return t2 - t0

        def driver():
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            return one("driver")

        def after_settle_3rd():  # the same settle, then the third launch+sync batch
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            one(None)
            one(None)
            return one("after_settle_3rd")

        def short_settle():  # 5 back-to-back batches instead of ~60 ms of them
            for _ in range(5):
                p.launch_steps(S, False, False)
            p.sync()
            return one("short_settle")

        def idle_1ms():  # the settle, then the GPU idle for 1 ms, then the batch
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            time.sleep(1e-3)
            return one(None)

        def rearm_idle(us):  # bench.py's re-arm batch, then the GPU idle for `us` (a host
            def fn():        # barrier's worth), then the batch
                for _ in range(settle):
                    p.launch_steps(S, False, False)
                p.sync()
                one(None)
                t_end = time.perf_counter() + us * 1e-6
                while time.perf_counter() < t_end:
                    pass
                return one(None)
            return fn

        def second():  # the settle, then the second launch+sync batch
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            one(None)
            return one("second")

        def devsync():  # the settle, the plan's sync and a device-wide sync (bench.py's order)
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            torch.cuda.synchronize()
            return one("devsync")

        def warm1():  # the settle, then one untimed 1-step batch (a single fused launch)
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            p.launch_steps(1, False, False)
            p.sync()
            return one("warm1")

        parts = {"launch": [], "sync": [], "device_sync": [], "idle_device_sync": []}

        def bench_like():  # bench.py's timed region after its re-arm batch, taken apart
            for _ in range(settle):
                p.launch_steps(S, False, False)
            p.sync()
            one(None)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.launch_steps(S, False, False)
            t1 = time.perf_counter()
            p.sync()
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            parts["launch"].append((t1 - t0) * 1e6)
            parts["sync"].append((t2 - t1) * 1e6)
            parts["device_sync"].append((t3 - t2) * 1e6)
            parts["idle_device_sync"].append((t4 - t3) * 1e6)
            return t3 - t0

        modes = [("back_to_back", back_to_back), ("synced", synced), ("driver", driver),
                 ("after_settle_3rd", after_settle_3rd), ("short_settle", short_settle),
                 ("idle_1ms", idle_1ms), ("second", second), ("devsync", devsync),
                 ("warm1", warm1), ("bench_like", bench_like)]
        if a.idle_us:
            modes = [("second", second)] + [(f"rearm_idle_{u}us", rearm_idle(u))
                                            for u in (int(x) for x in a.idle_us.split(","))]
        res.update({m: [] for m, _ in modes if m not in res})
        for r in range(a.reps):
            order = modes[r % len(modes):] + modes[:r % len(modes)]
            for name, fn in order:
                if name == "synced":  # as the tools run it: a few synced batches, the last one
                    for _ in range(5):
                        fn()
                res[name].append(fn() * 1e6)
        row = {"slice": g, "steps": S, "reps": a.reps, "grid": p.grid,
               **{f"{k}_us_median": statistics.median(v) for k, v in res.items() if v},
               **{f"{k}_us_min": min(v) for k, v in res.items() if v},
               **{f"{k}_launch_call_us_median": statistics.median(v)
                  for k, v in launch_call.items() if v},
               **{f"bench_like_{k}_us_median": statistics.median(v)
                  for k, v in parts.items() if v},
               "value": p.host_result(p.host_index_of(S - 1, False))}
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
