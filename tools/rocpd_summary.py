#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (its default output format).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db > profiles/r1/x.md

Prints a markdown table: kernel, calls, median/mean/min/max duration (us), share of GPU
time, grid, workgroup, VGPR/SGPR counts and LDS bytes (the launch resources the occupancy
analysis in docs/ARCHITECTURE.md relies on).
"""
from __future__ import annotations

import sqlite3
import statistics
import sys


def _strip_args(name: str) -> str:
    """`void f<(E)0, T>(args)` -> `f<(E)0, T>`: cut at the first '(' outside template brackets."""
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            return name[:i]
    return name


def summarize(path: str, top: int = 20) -> str:
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, duration, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, sgpr_count,"
        " lds_size from kernels").fetchall()
    by = {}
    for name, dur, gx, wx, vg, ag, sg, lds in rows:
        e = by.setdefault(name, {"d": [], "res": (gx, wx, vg, ag, sg, lds)})
        e["d"].append(dur / 1000.0)
    total = sum(sum(e["d"]) for e in by.values()) or 1.0
    out = ["| kernel | calls | median us | mean us | min us | max us | % time | grid | wg |"
           " vgpr | agpr | sgpr | lds B |", "|" + "---|" * 13]
    for name, e in sorted(by.items(), key=lambda kv: -sum(kv[1]["d"]))[:top]:
        d = e["d"]
        gx, wx, vg, ag, sg, lds = e["res"]
        short = _strip_args(name.replace("miint::(anonymous namespace)::", ""))
        out.append(f"| `{short[:90]}` | {len(d)} | {statistics.median(d):.1f} | "
                   f"{statistics.mean(d):.1f} | {min(d):.1f} | {max(d):.1f} | "
                   f"{100 * sum(d) / total:.1f} | {gx} | {wx} | {vg} | {ag} | {sg} | {lds} |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summarize(sys.argv[1]))
