#!/usr/bin/env python3
"""Time the materialised profile fill (interp_fill: 18e6 samples = 144 MB of stores) and the
array sum that re-reads it, back to back as cintegrate --materialize runs them, over many
launches. Run under `rocprofv3 --kernel-trace --stats` for per-kernel durations.

    python tools/interp_fill_probe.py [reps] [sum grids, e.g. 1024,2048]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    import torch

    from cuda_v_mpi_amd.ops import kernels

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    n = 18_000_000
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    for _ in range(20):
        kernels.interp_fill(n, out=y)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        kernels.interp_fill(n, out=y)
    ev[1].record()
    torch.cuda.synchronize()
    fill_us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    total = float(kernels.sum_array(y, scale=1e-4).item())
    print(json.dumps({"what": "interp_fill 18e6 samples (144 MB stores)", "reps": reps,
                      "us_per_fill": fill_us, "TB_per_s": n * 8 / (fill_us * 1e-6) / 1e12,
                      "distance": total}))
    # the re-read: sum_array (+ its finalize) over the same 144 MB at several grid sizes
    from cuda_v_mpi_amd import native

    m = native()
    out = torch.empty(1, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for grid in [int(g) for g in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1024"])]:
        parts = torch.empty(grid, dtype=torch.float64, device="cuda")
        for _ in range(20):
            m.launch_sum_array(y.data_ptr(), n, 1e-4, parts.data_ptr(), grid, out.data_ptr(), stream)
        ev[0].record()
        for _ in range(reps):
            m.launch_sum_array(y.data_ptr(), n, 1e-4, parts.data_ptr(), grid, out.data_ptr(), stream)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
        print(json.dumps({"what": "sum_array + finalize, 144 MB", "grid": grid, "reps": reps,
                          "us_per_sum": us, "TB_per_s": n * 8 / (us * 1e-6) / 1e12,
                          "distance": float(out.item())}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
