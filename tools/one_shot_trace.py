#!/usr/bin/env python3
"""One pi4 N = 1e9 integration per call, for a kernel trace of the settled one-shot
(`rocprofv3 --kernel-trace --stats -- python3 tools/one_shot_trace.py`): the plan the bench's
`single_shot_1e9` extra uses (multistep off: one fused launch per call whose last workgroup
stores the value into pinned memory), 400 settling calls and 50 timed ones of each form.
Prints the forms' medians as one JSON line.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from cuda_v_mpi_amd import Integrator

    it = Integrator("pi4", n=10**9, multistep=False)
    out = {"grid": it.plan.grid}
    for mode in ("direct_poll", "graph_poll"):
        r = it.plan.time_one_shot(50, mode, 400)
        out[mode] = {"median_us": r["median_us"], "device_median_us": r["device_median_us"]}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
