"""Probe: W loopback ranks driving RiemannPlans from Python threads, step by step.

    python tools/loopback_probe.py --world 2 --steps 37 [--graphs] [--stack-mb 64]

Prints a line per rank and phase (flushed), so a crash names the phase it happened in.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=37)
    ap.add_argument("--graphs", action="store_true")
    ap.add_argument("--prepare", action="store_true")
    ap.add_argument("--stack-mb", type=int, default=0)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    if a.stack_mb:
        threading.stack_size(a.stack_mb << 20)
    if not a.no_torch:
        import torch

        print("torch cuda", torch.cuda.is_available(), flush=True)
    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.parallel import loopback

    def body(rank, comm):
        it = Integrator("pi4", n=10**9, rule="mid", comm_obj=comm)
        p = it.plan
        print(f"rank {rank}: plan world={p.world} begin={p.begin}", flush=True)
        if a.prepare:
            p.prepare_steps(a.steps)
            print(f"rank {rank}: prepared ({p.graph_error!r})", flush=True)
        p.launch_steps(a.steps, True, a.graphs)
        print(f"rank {rank}: launched", flush=True)
        p.sync()
        v = p.host_result(p.host_index_of(a.steps - 1, a.graphs))
        print(f"rank {rank}: value {v!r} graph_launches {p.graph_launches}", flush=True)
        return v

    vals = loopback.run_ranks(a.world, body)
    print("values", vals, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
