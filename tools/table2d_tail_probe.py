#!/usr/bin/env python3
"""How much of a 2-D field launch is the fused last-workgroup tail?

Times, per launch (torch events around 200 back-to-back launches on one stream), the row
stream kernel with and without the in-kernel hand-off (slot publish + ticket + the last
workgroup's ordered read of every slot), for the whole 4096^2 / 8192^2 grid and one GPU's
1/8 row slice. Prints one JSON line per case.

    python tools/table2d_tail_probe.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cuda_v_mpi_amd import native  # noqa: E402
from cuda_v_mpi_amd.ops import kernels  # noqa: E402
from cuda_v_mpi_amd.utils import fixtures  # noqa: E402


def timed(fn, iters: int = 200) -> float:
    for _ in range(40):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main() -> None:
    m = native()
    v = torch.as_tensor(fixtures.profile_table(), device="cuda")
    T = kernels.outer_product(v)
    n = T.shape[0]
    s = torch.cuda.current_stream().cuda_stream
    for g in (4096, 8192):
        for r0, r1 in ((0, g), (3 * g // 8, 4 * g // 8)):
            nb = m.table2d_grid(n, n, 1800.0, 1800.0, g, g, r0, r1)
            parts = torch.empty(nb, dtype=torch.float64, device="cuda")
            m.fill_unset_slots(parts.data_ptr(), nb, s)
            ticket = torch.zeros(m.TICKET_WORDS, dtype=torch.int32, device="cuda")
            out = torch.zeros(1, dtype=torch.float64, device="cuda")
            fused = timed(lambda: m.launch_table2d_fused(T.data_ptr(), n, n, 1800.0, 1800.0, g, g,
                                                         r0, r1, parts.data_ptr(),
                                                         ticket.data_ptr(), out.data_ptr(), s))
            plain = timed(lambda: m.launch_table2d_partials(T.data_ptr(), n, n, 1800.0, 1800.0, g,
                                                            g, r0, r1, parts.data_ptr(), s))
            empty = timed(lambda: torch.cuda._sleep(0))
            print(json.dumps({"grid": g, "rows": [r0, r1], "workgroups": nb,
                              "path": m.table2d_path(n, n, 1800.0, 1800.0, g, g, r0, r1),
                              "fused_us": round(fused, 2), "partials_only_us": round(plain, 2),
                              "tail_us": round(fused - plain, 2),
                              "empty_launch_us": round(empty, 2)}), flush=True)


if __name__ == "__main__":
    main()
