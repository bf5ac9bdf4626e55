#!/usr/bin/env python3
"""Host API cost against device work, from a rocprofv3 runtime trace (CSV).

    rocprofv3 --runtime-trace --output-format csv -d OUT -o run -- python3 tools/batch_ab.py ...
    python tools/api_trace_summary.py OUT [--skip 0.5]

For every HIP API function: calls and median host duration. For every kernel and copy:
median device duration and the latency from the API call that enqueued it (matched by
correlation id: for a graph replay every node carries the hipGraphLaunch's id) to its start
on the device. --skip drops the first fraction of the run (warm-up, capture). Used for
profiles/r6/graph_vs_direct.md: where a graph replay of a multi-step batch spends the
microseconds a direct enqueue does not.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import sys


def _load(d: str, suffix: str) -> list[dict]:
    rows: list[dict] = []
    for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def _key(row: dict, *names: str) -> str:
    low = {k.lower(): k for k in row}
    for n in names:
        if n.lower() in low:
            return low[n.lower()]
    raise KeyError(names)


def summarize(d: str, skip: float = 0.5) -> dict:
    api = _load(d, "hip_api_trace.csv")
    ker = _load(d, "kernel_trace.csv")
    cpy = _load(d, "memory_copy_trace.csv")
    if not api:
        raise SystemExit(f"no hip_api_trace.csv under {d}")
    ks, ke = _key(api[0], "Start_Timestamp"), _key(api[0], "End_Timestamp")
    kf, kc = _key(api[0], "Function"), _key(api[0], "Correlation_Id")
    t0 = min(int(r[ks]) for r in api)
    t1 = max(int(r[ke]) for r in api)
    cut = t0 + skip * (t1 - t0)
    calls = {}
    by_corr = {}
    for r in api:
        s, e = int(r[ks]), int(r[ke])
        by_corr[r[kc]] = (r[kf], s)
        if s < cut:
            continue
        calls.setdefault(r[kf], []).append((e - s) / 1e3)
    out = {"api": {f: {"calls": len(v), "median_us": statistics.median(v)}
                   for f, v in sorted(calls.items(), key=lambda kv: -len(kv[1]))}}
    dev = {}
    for rows, kind in ((ker, "kernel"), (cpy, "copy")):
        if not rows:
            continue
        s_k, e_k = _key(rows[0], "Start_Timestamp"), _key(rows[0], "End_Timestamp")
        c_k = _key(rows[0], "Correlation_Id")
        n_k = _key(rows[0], "Kernel_Name") if kind == "kernel" else None
        for r in rows:
            s, e = int(r[s_k]), int(r[e_k])
            if s < cut:
                continue
            name = r[n_k][:60] if n_k else "copy"
            ent = dev.setdefault(name, {"dur": [], "lat": [], "via": {}})
            ent["dur"].append((e - s) / 1e3)
            via = by_corr.get(r[c_k])
            if via:
                ent["lat"].append((s - via[1]) / 1e3)
                ent["via"][via[0]] = ent["via"].get(via[0], 0) + 1
    out["device"] = {n: {"count": len(v["dur"]), "median_us": statistics.median(v["dur"]),
                         "launch_to_start_median_us": (statistics.median(v["lat"])
                                                       if v["lat"] else None),
                         "enqueued_by": v["via"]}
                     for n, v in dev.items()}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dir")
    ap.add_argument("--skip", type=float, default=0.5)
    a = ap.parse_args(argv)
    print(json.dumps(summarize(a.dir, a.skip), indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
