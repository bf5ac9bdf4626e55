"""W logical ranks on one GPU: the loopback transport (``_miint.LoopbackGroup``).

The reference's point is its P-rank decomposition (riemann.cpp:62-86 master/worker gather,
4main.c:95-221 distributed two-phase scan). RCCL refuses two ranks on one device, and the
test pool gives one GPU, so the production RCCL communicator can only ever run world = 1
there. The loopback communicator implements the same ``Comm`` interface (all-reduce,
all-gather, broadcast, reduce, group-wide graph capture) for W ranks on device 0, one host
thread per rank, so every world > 1 path of RiemannPlan, TrainScan and Table2DPlan runs
for real on the GPU: rank slicing, bucketed and per-step reductions, captured graphs,
rank carries fed by a real all-gather, parity windows, --replicate.

    from cuda_v_mpi_amd.parallel import loopback
    vals = loopback.run_ranks(8, lambda rank, comm: my_rank_body(rank, comm))

The native CLIs take ``--loopback W`` for the same thing.
"""
from __future__ import annotations

import threading
from typing import Any, Callable


def group(world: int, device: int = 0, timeout_s: float = 120.0):
    from .._native import native

    return native().LoopbackGroup(world, device, timeout_s)


def run_ranks(world: int, fn: Callable[[int, Any], Any], device: int = 0,
              timeout_s: float = 120.0) -> list:
    """Run ``fn(rank, comm)`` for every rank in its own thread; return the per-rank values.

    The native calls that synchronise ranks release the GIL. The first failure breaks the
    group (every other rank's next collective raises instead of waiting) and is re-raised.
    """
    grp = group(world, device, timeout_s)
    out: list = [None] * world
    errs: list = []

    def body(r: int) -> None:
        try:
            out[r] = fn(r, grp.comm(r))
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append((r, e))
            grp.mark_broken(f"rank {r} failed: {e}")

    th = [threading.Thread(target=body, args=(r,), name=f"loopback-rank-{r}")
          for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        r, e = min(errs, key=lambda x: "broken" in str(x[1]))  # root cause first
        raise RuntimeError(f"loopback rank {r}: {e}") from e
    run_ranks.last_group = grp  # type: ignore[attr-defined]
    return out
