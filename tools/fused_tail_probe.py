#!/usr/bin/env python3
"""Where the fused Riemann kernel's last ~2.6 us go (fused 76.2 us vs partials-only 73.6 us
at N = 1e9): run the headline plan with the result stored into mapped pinned host memory
(default) or into device memory (+ a copy node), for kernel-trace comparison.

    rocprofv3 --kernel-trace -d OUT -o run -- python3 tools/fused_tail_probe.py [--device-result]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cuda_v_mpi_amd._native import native  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device-result", action="store_true")
    ap.add_argument("--steps", type=int, default=960)
    a = ap.parse_args()
    m = native()
    cfg = m.RiemannConfig()
    cfg.integrand = m.Integrand.pi4
    cfg.a, cfg.b, cfg.n = 0.0, 1.0, 10**9
    cfg.slots = 48
    cfg.host_direct = not a.device_result
    plan = m.RiemannPlan(cfg, 0)
    t = plan.run_steps(a.steps, False, True)
    print({"host_direct": cfg.host_direct, "ms_per_step": t["device_ms"] / a.steps,
           "value": plan.host_result(0)}, flush=True)


if __name__ == "__main__":
    main()
