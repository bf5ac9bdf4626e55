#!/usr/bin/env python3
"""Headline benchmark: Riemann subintervals/s of 4/(1+x^2) on [0,1], N=1e9 fp64 per GPU.

Metric and config come from BASELINE.json ("Riemann subintervals/sec at N=1e9 fp64; |error|
vs analytic pi"). One step = one complete integration of N samples per GPU: gfx950 kernel
(every sample evaluated, fp64) -> in-kernel DPP/LDS/ticket reduction -> RCCL all-reduce of
the per-GPU partial over xGMI -> D2H into pinned memory. Steps are hipGraph replays of
batches of --slots (48) steps; with >1 GPU each batch ends in ONE all-reduce of its 48 step
results (bucketed: every step still gets its own global sum; --no-bucket = one 8-byte
all-reduce per step, overlapped on a side stream).

Warmup: the W warmup steps, then at least --settle-ms (60) more untimed steps so the timed
region starts at steady clocks (from idle the GPU ramps from ~90 to 76.8 us per step over
~25 ms; the JSON line reports the settle steps run as "warmup_settle_steps").

Weak scaling: every GPU integrates its own 1e9-sample slice of a global N = 1e9 x n_gpus
(N = 8e9 on 8 GPUs). The results of the last batch of timed steps (every rank holds the
global sums) are checked on the host against pi.

    python bench.py                          # 1 GPU
    torchrun --nproc-per-node 8 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# Reference CPU number for the same metric/config (4/(1+x^2), N=1e9, left rule,
# 8 Xeon workers, -O2): 0.203 s -> 4.94e9 subintervals/s, |err| 1.000e-9.
BASELINE_SUBINT_PER_S = 4.94e9


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--settle-ms", type=float, default=60.0,
                   help="after the W warmup steps, keep stepping (untimed) for at least this "
                        "long so the timed steps run at steady clocks (0 = off)")
    # (--n is a prefix of torchrun's own --nnodes/--nproc-per-node: use --samples under torchrun)
    p.add_argument("--samples", "--n", dest="n", type=float, default=1e9,
                   help="samples per GPU (weak) or total (strong)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--integrand", default="pi4")
    p.add_argument("--rule", default="left", choices=["left", "mid", "right"])
    p.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    p.add_argument("--div", default="series", choices=["series", "ieee", "series_direct"])
    p.add_argument("--comm", default="native", choices=["native", "torch"],
                   help="native: C++ RCCL communicator captured in the step graph; "
                        "torch: torch.distributed all_reduce of each step's partial")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend (gloo only for functional tests on shared GPUs)")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-pipeline", action="store_true")
    p.add_argument("--unfused", action="store_true", help="partials + finalize (2 launches)")
    p.add_argument("--grid", type=int, default=0)
    p.add_argument("--slots", type=int, default=48,
                   help="steps per captured graph batch (= steps per bucketed all-reduce)")
    p.add_argument("--no-bucket", action="store_true",
                   help="one all-reduce per step instead of one per graph batch of steps")
    p.add_argument("--force-collective", action="store_true",
                   help="run the RCCL all-reduce stage even on 1 GPU (tests the multi-GPU graph)")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--jsonl", default="", help="also append the JSON line to this file")
    return p.parse_args()


def main() -> int:
    args = parse()
    import torch
    import torch.distributed as dist

    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.parallel import dist as mdist

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        if world_env == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} needs torchrun with {args.gpus} processes",
                  file=sys.stderr)
            return 2
    if args.backend == "gloo" and args.comm == "native" and world_env > 1:
        print("bench.py: --backend gloo shares GPUs between ranks; use --comm torch", file=sys.stderr)
        return 2
    ctx = mdist.init(backend=args.backend)
    world = ctx.world
    n_per = int(args.n)
    n_total = n_per * world if args.scaling == "weak" else n_per

    use_torch = args.comm == "torch" and world > 1
    integ = Integrator(args.integrand, n=n_total, rule=args.rule, dtype=args.dtype, div=args.div,
                       backend="hip", ctx=ctx, comm=args.comm, fused=not args.unfused,
                       grid=args.grid, slots=args.slots, force_collective=args.force_collective,
                       bucket=not args.no_bucket)
    plan = integ.plan
    graphs = not args.no_graph and not use_torch
    pipeline = not args.no_pipeline and (world > 1 or args.force_collective)

    if use_torch:  # kernels on the torch stream + torch.distributed all_reduce per step
        from cuda_v_mpi_amd.parallel.torch_steps import TorchStepper

        stepper = TorchStepper(integ.spec, n_total, ctx, rule=args.rule, dtype=args.dtype,
                               div=args.div, grid=args.grid or None)
        launch, finish, result = stepper.launch_steps, stepper.sync, stepper.result
    else:
        launch = lambda k: plan.launch_steps(k, pipeline, graphs)  # noqa: E731
        finish = plan.sync
        result = lambda k: plan.host_result(plan.host_index_of(k, graphs))  # noqa: E731

    # ---- warmup (includes graph capture and RCCL channel setup)
    launch(max(1, args.warmup))
    finish()
    if graphs and not plan.graphs_ready:
        print(f"bench.py: hipGraph capture failed ({plan.graph_error}); "
              "running with direct stream enqueue", file=sys.stderr)
        graphs = False
    # ---- clock settle: from idle the MI355X needs ~25 ms of continuous work before its
    # per-step time is steady (90 -> 76.8 us per step; profiles/r1/clock_ramp.jsonl). The W
    # warmup steps alone (20 x 85 us) end inside that ramp, so the warmup also runs at least
    # --settle-ms of back-to-back steps. The step count comes from one calibration batch,
    # agreed across ranks (MAX) so every rank runs the same collectives.
    settle_steps = 0
    if args.settle_ms > 0:
        t_c = time.perf_counter()
        launch(plan.slots)
        finish()
        per_step = (time.perf_counter() - t_c) / plan.slots
        want = torch.tensor([math.ceil(args.settle_ms * 1e-3 / max(per_step, 1e-7))],
                            dtype=torch.float64, device="cuda" if ctx.backend == "nccl" else "cpu")
        ctx.all_reduce_max(want)
        settle_steps = plan.slots + int(want.item())
        launch(settle_steps - plan.slots)
        finish()

    # ---- timed region: barrier + device sync on both sides, K steps in between
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch(args.steps)
    finish()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.barrier()
    elapsed = t1 - t0

    t = torch.tensor([elapsed], dtype=torch.float64,
                     device="cuda" if ctx.backend == "nccl" else "cpu")
    ctx.all_reduce_max(t)
    elapsed_max = float(t.item())

    # ---- verify the results of the last steps (every rank holds the global value)
    analytic = integ.spec.analytic()
    last = range(max(0, args.steps - min(args.steps, plan.slots)), args.steps)
    vals = [result(k) for k in last]
    errs = [abs(v - analytic) for v in vals]
    abs_err = max(errs)
    # left rule truncation for 4/(1+x^2) is exactly h; anything far above is a bug
    tol = 4.0 * (integ.spec.b - integ.spec.a) / n_total + 1e-12 if args.rule == "left" else 1e-9
    ok = all(math.isfinite(v) for v in vals) and (args.dtype != "fp64" or abs_err <= tol)

    ms_per_step = elapsed_max / args.steps * 1e3
    value = n_total * args.steps / elapsed_max
    if ctx.is_root:
        out = {
            "metric": "Riemann subintervals/sec at N=1e9 fp64; |error| vs analytic pi",
            "value": value,
            "unit": "subintervals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_settle_steps": settle_steps,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": value / BASELINE_SUBINT_PER_S,
            "dtype": args.dtype,
            "data": "synthetic (analytic integrand 4/(1+x^2); no dataset)",
            "abs_err": abs_err,
            "result": vals[-1],
            "verified": ok,
            "config": {
                "model": f"riemann_{args.integrand}_{args.dtype}",
                "integrand": "4/(1+x^2) on [0,1]" if args.integrand == "pi4" else args.integrand,
                "N": n_total,
                "n_per_gpu": n_total // world if args.scaling == "weak" else n_total // world,
                "rule": args.rule,
                "division": str(plan.effective_div).split(".")[-1],
                "global_batch": n_total,
                "seq_len": 1,
                "parallelism": f"dp{world}",
                "comm": args.comm if (world > 1 or args.force_collective) else "none",
                "graphs": graphs,
                "graph_nodes": plan.graph_nodes if graphs else 0,
                "pipeline": pipeline,
                "bucketed_allreduce": bool(plan.bucketed),
                "fused_reduction": not args.unfused,
                "chained_batches": bool(plan.chained) and graphs,
                "grid": plan.grid,
            },
        }
        print(json.dumps(out), flush=True)
        if args.jsonl:
            with open(args.jsonl, "a") as f:
                f.write(json.dumps(out) + "\n")
    ctx.destroy()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
