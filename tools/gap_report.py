#!/usr/bin/env python3
"""Kernel gaps of the timed region from a rocprofv3 kernel trace (CSV or rocpd database).

    rocprofv3 --kernel-trace [--output-format csv] -d OUT -o run -- python3 bench.py --steps 20 --warmup 5 --no-extras
    python tools/gap_report.py OUT --last 21

Prints the last `--last` dispatches (the timed region of a bench.py run is its final graph
replay: K chained kernels + the finalize closing the batch), each kernel's duration and the
idle gap since the previous one ended, plus totals.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sqlite3
import statistics


def _rows(d: str) -> list[dict]:
    """Dispatches as CSV-style dicts, from the CSV trace files or, failing those, from the
    rocpd SQLite databases (rocprofv3's default output format)."""
    rows: list[dict] = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    if rows:
        return rows
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        db = sqlite3.connect(f)
        try:
            rows.extend({"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                        for n, s, e in db.execute("select name, start, end from kernels"))
        finally:
            db.close()
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=21)
    a = ap.parse_args()
    rows = _rows(a.dir)
    if not rows:
        print(f"no kernel dispatches under {a.dir} (*kernel_trace.csv or *_results.db)")
        return 1
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-a.last:]
    prev_end = None
    gaps, durs = [], []
    for r in tail:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = None if prev_end is None else (s - prev_end) / 1e3
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("miint::", "")
        name = name.replace("void ", "").split("(miint")[0].split("(RiemannParams")[0][:70]
        print(f"{name:72s} {(e - s) / 1e3:9.2f} us  gap {'' if gap is None else f'{gap:7.2f} us'}")
        if gap is not None:
            gaps.append(gap)
        durs.append((e - s) / 1e3)
        prev_end = e
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    print(f"span {span:.1f} us over {len(tail)} dispatches; kernel time {sum(durs):.1f} us; "
          f"gaps: max {max(gaps):.2f} us, median {statistics.median(gaps):.2f} us, "
          f"sum {sum(gaps):.2f} us")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
