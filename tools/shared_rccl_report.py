#!/usr/bin/env python3
"""Summary of tools/shared_gpu_rccl.sh: W RCCL ranks sharing ONE GPU against one rank.

    python tools/shared_rccl_report.py gpurun_out/shared_rccl/records.jsonl > summary.md

Every multi-rank record is the slowest rank's time behind a collective barrier, so W ranks
on one GPU may not report more than that GPU's single-rank rate of the same tool: the
`<= np1` column checks it (rate = samples per second of the timed work; 2 % slack for
run-to-run noise). The transport columns are what RCCL's INIT log says (NET/Socket with
nNodes = W: every rank presents itself as a host of its own).
"""
from __future__ import annotations

import json
import sys

SLACK = 1.02


def rate(r: dict) -> float | None:
    if "subintervals_per_s" in r:
        return r["subintervals_per_s"]
    if r.get("program") == "cintegrate" and r.get("device_ms"):
        return 18e6 / (r["device_ms"] * 1e-3)
    if r.get("program") == "trainscan" and r.get("device_ms"):
        return 18e6 / (r["device_ms"] * 1e-3)
    if r.get("program") == "table2d" and r.get("ms_per_integration"):
        return r["grid"] ** 2 / (r["ms_per_integration"] * 1e-3)
    if "metric" in r:  # bench.py
        return r["value"]
    return None


def base_of(step: str) -> str:
    for suf in ("_np1", "_np2", "_np3", "_np4", "_np8"):
        if step.endswith(suf):
            return step[: -len(suf)]
    return step


def main() -> int:
    recs = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
    # one row per step (miint comm prints one record per op x size: keep its first, the 8-B
    # all-reduce)
    seen, rows = set(), []
    for r in recs:
        if r["step"].startswith("miint_comm"):
            if r["step"] in seen:
                continue
        seen.add(r["step"])
        rows.append(r)
    recs = rows
    one = {base_of(r["step"]): rate(r) for r in recs if r["step"].endswith("_np1") and rate(r)}
    one.setdefault("bench_torch", one.get("bench_native"))  # the same config, other data plane
    print("| step | ranks | comm | rccl_world | transport | nNodes | share GPU | rate /s | "
          "np1 rate /s | <= np1 |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    bad = 0
    for r in recs:
        step = r["step"]
        ranks = r.get("gpus", r.get("n_gpus", 1))
        rt = rate(r)
        ref = one.get(base_of(step).replace("bench_strong", "bench_native"))
        ok = "" if ranks == 1 or rt is None or ref is None or "parity" in step else (
            "yes" if rt <= SLACK * ref else "**NO**")
        bad += ok == "**NO**"
        print(f"| {step} | {ranks} | {r.get('comm', r.get('control_plane', ''))} | "
              f"{r.get('rccl_world')} | {r.get('rccl_transport')} | {r.get('rccl_nnodes')} | "
              f"{r.get('ranks_share_gpus')} | {rt if rt is None else f'{rt:.4g}'} | "
              f"{'' if ref is None else f'{ref:.4g}'} | {ok} |")
    print()
    print(f"multi-rank records above their tool's one-rank rate: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
