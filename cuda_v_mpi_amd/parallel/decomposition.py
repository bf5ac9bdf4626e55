"""Domain decomposition: which samples each rank owns.

Reference strategies:
  P1  riemann.cpp:65-86   master/worker: rank 0 idles, worker w gets [w R/W, (w+1) R/W) with
                          (int)(N/W) samples — P=1 yields 0, N%W samples are dropped.
  P2  4main.c:76-78,90-91 SPMD: fill partition by whole seconds, scan partition by elements,
                          residual never scanned.
  P3  cintegrate.cu:48-59 one fat thread per contiguous chunk (64 threads per GPU).
The framework's own decomposition is `rank_slice`: a balanced 64-bit split of the global
sample index range where every rank (rank 0 included) works and nothing is dropped; the
reference partitions are kept for --parity emulation.
"""
from __future__ import annotations

import math


def rank_slice(n: int, rank: int, world: int) -> tuple[int, int]:
    """(begin, count) of rank's share of [0, n); first n % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, rem = divmod(n, world)
    count = q + (1 if rank < rem else 0)
    begin = rank * q + min(rank, rem)
    return begin, count


def master_worker_slices(comm_size: int, n: float, rng: float = math.pi):
    """riemann.cpp partition: list of (left, right, local_n) per worker (rank 1..P-1)."""
    workers = comm_size - 1
    out = []
    for w in range(workers):
        left = w * (rng / workers)
        out.append((left, left + rng / workers, int(n / workers)))
    return out


def trainscan_partitions(comm_size: int, seconds: int = 1800, steps_per_sec: int = 10000):
    """4main.c partitions per rank: (fill_lo, fill_hi, scan_lo, scan_hi) element ranges."""
    T = seconds * steps_per_sec
    fs = (seconds // comm_size) * steps_per_sec
    sub = T // comm_size
    return [(r * fs, r * fs + fs, r * sub, r * sub + sub) for r in range(comm_size)]


def cintegrate_chunks(sp: int, sm: int, seconds: int = 1800, steps_per_sec: int = 10000):
    """cintegrate.cu:79-82 per-thread element chunks [lo, hi)."""
    w = sp * sm
    chunk = seconds // w
    return [(r * chunk * steps_per_sec, (r + 1) * chunk * steps_per_sec) for r in range(w)]


def coverage_seconds(workers: int, seconds: int = 1800) -> int:
    """Seconds actually integrated when each of `workers` gets floor(seconds/workers)."""
    return (seconds // workers) * workers
