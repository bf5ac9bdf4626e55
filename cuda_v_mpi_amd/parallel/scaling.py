"""GPU-count scaling sweep (SURVEY §7.1 layer 10): the headline over N in {1, 2, 4, 8} GPUs.

The reference measures its decomposition by re-running ``mpirun -np P`` by hand
(riemann.cpp:62-86, 4main.c:69-157) and reading a wall clock. Here one command runs, for
every GPU count the node has,

  * ``bench.py --gpus N`` (one process per GPU, spawned by bench.py itself; RCCL over xGMI):
    the headline, which is the metric's own config at every N (N = 1e9 samples IN TOTAL over
    the N GPUs, as the reference splits its fixed STEPS over its workers,
    riemann.cpp:10,71-73: strong scaling) and, from the same run, the weak form
    (``weak_1e9_per_gpu``: 1e9 samples per GPU), BASELINE #3's strong-scaling point (N = 1e10
    in total) and BASELINE #5's 2-D field (4096^2 samples in total, rows split over the N
    GPUs);
  * ``miint comm --gpus N`` (one process driving N GPUs, ncclCommInitAll): all-reduce and
    all-gather latency at 8 B (the Riemann payload, riemann.cpp:76) and 144 MB (4main.c:157's
    broadcast table),

and derives strong- (the headline ``value``) and weak-scaling efficiency against the N = 1
row. Counts the node
cannot run get an explicit ``skipped`` row instead of a number.

    python -m cuda_v_mpi_amd scale --gpus 1,2,4,8 [--steps 200] [--jsonl FILE] [--md FILE]
    python bench.py --sweep-gpus 1,2,4,8

This process never touches the GPU (children do): the device count comes from
``torch.cuda.device_count()``, which does not initialise HIP on this stack.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BENCH = os.path.join(REPO, "bench.py")
MIINT = os.path.join(REPO, "build", "bin", "miint")


def visible_gpus() -> int:
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover - no torch / no ROCm
        return 0


def _last_json(text: str) -> dict | None:
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def run_bench(n: int, steps: int, warmup: int, timeout: float = 900.0,
              extra: list[str] | None = None) -> dict:
    cmd = [sys.executable, BENCH, "--gpus", str(n), "--steps", str(steps), "--warmup",
           str(warmup)] + list(extra or [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    js = _last_json(p.stdout)
    if p.returncode != 0 or js is None:
        raise RuntimeError(f"bench.py --gpus {n} failed (rc {p.returncode}): {p.stderr[-2000:]}")
    return js


def run_comm(n: int, timeout: float = 600.0) -> dict:
    """8 B and 144 MB all-reduce / all-gather times (slowest rank) from `miint comm`."""
    if not os.path.exists(MIINT):
        return {"skipped": f"{MIINT} not built"}
    p = subprocess.run([MIINT, "comm", "--gpus", str(n), "--max-bytes", "144e6", "--iters", "10"],
                       capture_output=True, text=True, timeout=timeout, cwd=REPO)
    if p.returncode != 0:
        return {"error": p.stderr[-1000:]}
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    out = {}
    if rows:  # the transport the sweep's collectives used (one process, n devices)
        out["comm_rccl_transport"] = rows[0].get("rccl_transport")
    for r in rows:
        b = r["bytes"] / (n if r["op"] == "allgather" else 1)  # per-rank payload
        if r["op"] in ("allreduce", "allgather") and (b == 8 or b >= 144e6 * 0.99):
            key = f"{r['op']}_{'8B' if b == 8 else '144MB'}"
            out[key + "_us"] = r["us"]
            out[key + "_busbw_GBps"] = r["busbw_GBps"]
    return out


def sweep(counts: list[int], steps: int = 200, warmup: int = 10, comm: bool = True) -> list[dict]:
    """One row per GPU count. Under MIINT_OVERSUBSCRIBE=1 (``dist.ranks_share_devices``) a
    count above the visible devices still runs, its ranks sharing GPUs over RCCL's loopback
    sockets: a rehearsal of the sweep's multi-rank path, marked ``ranks_share_gpus`` and given
    no efficiency (the GPUs are time-shared, so the numbers say nothing about scaling)."""
    from .dist import ranks_share_devices

    have = visible_gpus()
    shared = ranks_share_devices()
    rows: list[dict] = []
    for n in counts:
        if n > have and not (shared and have >= 1):
            rows.append({"n_gpus": n, "skipped": f"only {have} devices"})
            continue
        b = run_bench(n, steps, warmup)
        row = {
            "n_gpus": n,
            "value": b["value"],
            "ms_per_step": b["ms_per_step"],
            "per_rank_spread_ms": b.get("per_rank_spread_ms"),
            "rccl_world": b.get("rccl_world"),
            "rccl_version": b.get("rccl_version"),
            # what RCCL's INIT log says the ranks' connections use (P2P/IPC over xGMI on one
            # node), and the record's verdict on it (bench.transport_check)
            "rccl_transport": b.get("rccl_transport"),
            "rccl_nnodes": b.get("rccl_nnodes"),
            "transport_error": b.get("transport_error"),
            "graphs": b["config"]["graphs"],
            # how a batch was launched: one persistent multi-step launch + close enqueued
            # directly (the default), or a graph replay
            "batch_launch": b["config"].get("batch_launch"),
            "verified": b["verified"],
        }
        if n > have:
            row["ranks_share_gpus"] = True
        # the headline is the metric's fixed N = 1e9 (strong); a record from --scaling weak
        # names its strong point "strong_1e9" and carries the weak figure at the top
        strong = b.get("scaling", "strong") == "strong"
        if not strong and b.get("strong_1e9"):
            w = {"value": b["value"], "ms_per_step": b["ms_per_step"], "verified": b["verified"]}
            row.update(value=b["strong_1e9"]["value"], ms_per_step=b["strong_1e9"]["ms_per_step"])
        else:
            w = b.get("weak_1e9_per_gpu")
        if w:
            row["weak_1e9_value"] = w["value"]
            row["weak_1e9_ms"] = w["ms_per_step"]
            row["weak_1e9_verified"] = w.get("verified")
        s = b.get("baseline3_strong_1e10")
        if s:
            row["strong_1e10_value"] = s["value"]
            row["strong_1e10_ms"] = s["ms_per_step"]
        t2 = b.get("baseline5_table2d_4096")
        if t2:
            row["t2d_4096_us"] = t2["ms_per_integration"] * 1e3
        one = b.get("single_shot_1e9")
        if one:
            row["one_shot_1e9_us"] = one["ms_one_shot"] * 1e3
        if comm and n <= have:  # miint comm drives n distinct devices from one process
            row.update(run_comm(n))
        rows.append(row)
    base = next((r for r in rows if r["n_gpus"] == 1 and "value" in r), None)
    for r in rows:
        if base is None or "value" not in r or r.get("ranks_share_gpus"):
            continue
        n = r["n_gpus"]
        r["strong_1e9_eff"] = r["value"] / (n * base["value"])  # the metric's own N
        if "weak_1e9_value" in r and "weak_1e9_value" in base:
            r["weak_eff"] = r["weak_1e9_value"] / (n * base["weak_1e9_value"])
        if "strong_1e10_value" in r and "strong_1e10_value" in base:
            r["strong_eff"] = r["strong_1e10_value"] / (n * base["strong_1e10_value"])
        if "t2d_4096_us" in r and "t2d_4096_us" in base:  # fixed total work: strong
            r["t2d_strong_eff"] = base["t2d_4096_us"] / (n * r["t2d_4096_us"])
    return rows


def markdown(rows: list[dict]) -> str:
    cols = ["n_gpus", "value", "ms_per_step", "strong_1e9_eff", "weak_1e9_value", "weak_1e9_ms",
            "weak_eff", "strong_1e10_value", "strong_eff",
            "t2d_4096_us", "t2d_strong_eff", "one_shot_1e9_us", "per_rank_spread_ms", "rccl_world",
            "rccl_transport", "rccl_nnodes", "allreduce_8B_us", "allgather_8B_us",
            "allreduce_144MB_us", "allgather_144MB_us"]
    out = ["| " + " | ".join(cols) + " |", "|" + "---|" * len(cols)]
    for r in rows:
        if "skipped" in r:
            out.append(f"| {r['n_gpus']} | skipped: {r['skipped']} |" + " |" * (len(cols) - 2))
            continue
        cells = []
        for c in cols:
            v = r.get(c)
            cells.append("" if v is None else (f"{v:.4g}" if isinstance(v, float) else str(v)))
        out.append("| " + " | ".join(cells) + " |")
    return "\n".join(out)


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-comm", action="store_true")
    ap.add_argument("--jsonl", default="")
    ap.add_argument("--md", default="")
    a = ap.parse_args(argv)
    rows = sweep([int(x) for x in a.gpus.split(",")], a.steps, a.warmup, comm=not a.no_comm)
    for r in rows:
        print(json.dumps(r), flush=True)
    md = markdown(rows)
    print(md)
    if a.jsonl:
        with open(a.jsonl, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    if a.md:
        with open(a.md, "w") as f:
            f.write(md + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
