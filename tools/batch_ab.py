#!/usr/bin/env python3
"""Interleaved A/B of batch variants on one GPU: the same per-GPU share, several plan options.

Separate runs of one variant after another drift with the clock state of the box (the same
20-step batch at the 1/8 share measured 191-200 us from run to run, profiles/r6/batch_tail.md),
so this tool builds every variant's plan first and then times them in rounds, one batch of
each variant per round, in rotating order: every variant sees the same drift. Per variant it
reports the median and minimum over rounds of the host time around one batch
(RiemannPlan.run_steps: launch call to results in pinned memory, the plan's own sync) and of
its hipEvent span, and checks that all variants gave the same value bit for bit.

    python tools/batch_ab.py --slice 8 --steps 20 \
        --variant close=kernel --variant close=launch [--collective] [--jsonl FILE]

A variant is comma-separated Integrator keywords (close=launch,allreduce_to_host=0,...);
graphs=1 / graphs=0 in a variant sets how that variant's batches run (else --graphs).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_variant(text: str) -> dict:
    kw: dict = {}
    for item in filter(None, text.split(",")):
        k, v = item.split("=", 1)
        if v.lower() in ("0", "false", "off", "no"):
            kw[k] = False
        elif v.lower() in ("1", "true", "on", "yes"):
            kw[k] = True
        else:
            try:
                kw[k] = int(v)
            except ValueError:
                kw[k] = v
    return kw


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--n", type=float, default=1e9, help="samples in total")
    ap.add_argument("--slice", type=int, default=1, help="rank 0's share of G GPUs")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--slots", type=int, default=48)
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--integrand", default="pi4")
    ap.add_argument("--collective", action="store_true", help="the 1-rank RCCL stage")
    ap.add_argument("--graphs", action="store_true", help="batches as graph replays")
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--values-may-differ", action="store_true",
                    help="variants that change the summation (block size, grid): report "
                         "values without failing on a difference")
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)

    from cuda_v_mpi_amd import Integrator

    variants = a.variant or [""]
    plans = []
    graphs_of = {}
    for text in variants:
        vk = parse_variant(text)
        name = text or "default"
        graphs_of[name] = bool(vk.pop("graphs", a.graphs))
        kw = dict(n=int(a.n), slots=a.slots, force_collective=a.collective,
                  slice_of=(0, a.slice))
        kw.update(vk)  # a variant may set any of these too (force_collective=1, ...)
        it = Integrator(a.integrand, **kw)
        if graphs_of[name]:
            it.plan.prepare_steps(a.steps)
        plans.append((name, it))
    # warm: >= 30 ms of each variant's batches (code objects, RCCL, clocks)
    for name, it in plans:
        for _ in range(max(1, math.ceil(0.03 / 2e-4 / a.steps))):
            it.plan.run_steps(a.steps, a.collective, graphs_of[name])
    host = {name: [] for name, _ in plans}
    dev = {name: [] for name, _ in plans}
    for r in range(a.rounds):
        order = plans[r % len(plans):] + plans[:r % len(plans)]
        for name, it in order:
            t = it.plan.run_steps(a.steps, a.collective, graphs_of[name])
            host[name].append(t["wall_s"] * 1e6)
            dev[name].append(t["device_ms"] * 1e3)
    values = {name: it.plan.host_result(it.plan.host_index_of(a.steps - 1, graphs_of[name]))
              for name, it in plans}
    same = len(set(values.values())) == 1
    rows = []
    for name, it in plans:
        h, d = host[name], dev[name]
        row = {"variant": name, "slice": a.slice, "n_per_gpu": it.plan.count,
               "grid": it.plan.grid, "steps": a.steps, "rounds": a.rounds,
               "collective": a.collective, "graphs": graphs_of[name],
               "graph_nodes": it.plan.graph_nodes,
               "close_in_launch": it.plan.close_in_launch,
               "allreduce_to_host": it.plan.allreduce_to_host,
               "host_us_median": statistics.median(h), "host_us_min": min(h),
               "host_us_per_step_median": statistics.median(h) / a.steps,
               "device_us_median": statistics.median(d), "device_us_min": min(d),
               "value": values[name], "values_bitwise_equal": same}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for row in rows:
                f.write(json.dumps(row) + "\n")
    return 0 if (same or a.values_may_differ) else 1


if __name__ == "__main__":
    sys.exit(main())
