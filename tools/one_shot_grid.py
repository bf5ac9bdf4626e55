#!/usr/bin/env python3
"""One-shot latency (launch -> pinned result, RiemannPlan.time_one_shot) of pi4 N = 1e9 fp64
against the launch grid and block: the single-integration form pays the launch ramp and the
tail of its last tile round in full, so its best grid need not be the multi-step one.

    python tools/one_shot_grid.py [reps] [mode] [warmup] -> one JSON line per (block, grid)

Each configuration runs `warmup` untimed calls first (default 400: from idle the clock needs
~250 single calls to settle, profiles/r4/oneshot_trace.md; round 4's first sweep used 30 and
is unsettled).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    mode = sys.argv[2] if len(sys.argv) > 2 else "direct_poll"
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    from cuda_v_mpi_amd import Integrator

    for block, grids in ((256, (0, 1024, 1536, 1792, 2048, 2304, 2560, 3072, 4096)),
                         (512, (0, 512, 768, 896, 1024)), (1024, (0, 256, 448, 512))):
        for g in grids:
            it = Integrator("pi4", n=10**9, multistep=False, grid=g, block=block)
            r = it.plan.time_one_shot(reps, mode, warmup)
            r.update(block=block, grid=it.plan.grid, grid_arg=g)
            print(json.dumps(r), flush=True)
            del it
    return 0


if __name__ == "__main__":
    sys.exit(main())
