"""Python command line: ``python -m cuda_v_mpi_amd <command> [flags]``.

Mirrors the native tools in build/bin (same stdout contract as the reference programs,
SURVEY §2.6) on top of the Python API, and adds JSON output:

    riemann     sin on [0, pi], N = 1e9 (riemann.cpp)          [--integrand pi4 --n 1e9 ...]
    cintegrate  train distance from the profile (cintegrate.cu)  [--parity --sp 32 --sm 2]
    trainscan   two-phase prefix scan (4main.c)                   [--parity --algo lookback]
    integrate   any integrand, JSON result                        [--integrand --n --rule ...]
                or any f(x):  --expr "exp(-x*x)" --a 0 --b 3 (compiled at run time, hipRTC)
    table2d     2-D velocity field v(x) v(y), bilinear, JSON      [--grid 4096 --iters 100]
    oracle      print every SURVEY §6.1 oracle value (CPU only)
    scale       GPU-count sweep 1,2,4,8: weak/strong efficiency, RCCL latency [--gpus 1,2,4,8]
    compare     the reference's CUDA-vs-MPI comparison, measured here: the same integral on
                the MI355X and on this host's cores (host engine; for sin also the reference's
                own scalar MPI program on threads)        [--integrand sin --n 1e9 --ranks 8]
    info        devices and build

Multi-GPU: launch under torchrun (one process per GPU); the process group is created from
the environment and partial sums are reduced with RCCL.
"""
from __future__ import annotations

import argparse
import json
import math
import sys

from .utils import output


def _elapsed() -> float:
    """Seconds since this process started (the reference starts its clock first thing in
    main(), before MPI_Init / context creation: riemann.cpp:51, cintegrate.cu:104)."""
    import time

    import psutil

    return time.time() - psutil.Process().create_time()


def _ctx(backend=None):
    """Process group for the ranks (torchrun env). GPU runs reduce through the native RCCL
    communicator, so their torch group is the gloo control plane (one RCCL communicator per
    rank); host/cpu backends reduce over gloo itself."""
    from .parallel import dist as mdist

    return mdist.init(backend=backend or mdist.control_backend("native"))


def cmd_riemann(a) -> int:
    from . import Integrator

    ctx = _ctx("gloo" if a.backend in ("cpu", "host") else None)
    spec_b = {"sin": math.pi, "pi4": 1.0}.get(a.integrand, None)
    it = Integrator(a.integrand, n=int(a.n), rule=a.rule, dtype=a.dtype, div=a.div, ctx=ctx,
                    backend=a.backend, block=a.block)
    r = it.run()
    if ctx.is_root:
        print(output.fmt_seconds(_elapsed()))
        print(output.fmt_riemann_result(spec_b if spec_b is not None else it.spec.b, a.n, r.value))
        if a.json:
            print(json.dumps(r.as_dict()))
    ctx.destroy()
    return 0


def cmd_cintegrate(a) -> int:
    from . import Integrator
    from .parallel.decomposition import coverage_seconds

    ctx = _ctx("gloo" if a.backend in ("cpu", "host") else None)
    seconds = coverage_seconds(a.sp * a.sm) if a.parity else 1800
    it = Integrator("table", n=seconds * 10000, rule="left", b=float(seconds), ctx=ctx,
                    backend=a.backend)
    r = it.run()
    if ctx.is_root:
        print(output.fmt_seconds(_elapsed()))
        print(output.fmt_cintegrate_distance(r.value))
        if a.json:
            print(json.dumps(r.as_dict()))
    ctx.destroy()
    return 0


def cmd_trainscan(a) -> int:
    from ._native import native
    from .parallel.dist import native_comm

    ctx = _ctx()
    m = native()
    cfg = m.TrainScanConfig()
    cfg.parity, cfg.algo = a.parity, a.algo
    comm = native_comm(ctx) if ctx.world > 1 else None
    if ctx.is_root:
        print(output.fmt_step_size(cfg.steps_per_sec))
    r = m.TrainScan(cfg, ctx.device, comm).run()
    if ctx.is_root:
        print(output.fmt_seconds(_elapsed()))
        print(output.fmt_total_distance(r["distance"]))
        if a.json:
            print(json.dumps(r))
    ctx.destroy()
    return 0


def cmd_compare(a) -> int:
    """The reference is a CUDA-vs-MPI comparison (its name; riemann.cpp vs cintegrate.cu):
    one JSON row per side, measured in this process, plus the ratio."""
    import time

    from . import Integrator
    from ._native import native

    m = native()
    n = int(a.n)
    rows = []

    def timed(fn, reps):
        fn()  # warm: threads, code, clocks
        best, v = float("inf"), None
        for _ in range(reps):
            t = time.perf_counter()
            v = fn()
            best = min(best, time.perf_counter() - t)
        return v, best

    if a.expr:  # any f(x): compiled for the host cores and, below, with hipRTC for gfx950
        lo = 0.0 if a.a is None else a.a
        hi = 1.0 if a.b is None else a.b
        pool = m.HostPool(a.threads)
        he = m.HostExpr(a.expr)
        rl = getattr(m.Rule, a.rule)
        v, s = timed(lambda: he.integrate(lo, hi, n, rl, 0, n, pool), a.reps)
        rows.append({"side": "host", "what": f"{a.expr} compiled for the host, "
                     f"{pool.threads} threads, scalar libm per sample", "value": v,
                     "seconds": s, "subintervals_per_s": n / s})
    else:
        host = Integrator(a.integrand, n=n, rule=a.rule, backend="host", threads=a.threads)
        v, s = timed(lambda: host.run().value, a.reps)
        rows.append({"side": "host", "what": f"host engine, {host._pool.threads} threads, "
                     f"{m.host_isa()}, per-sample fp64", "value": v,
                     "abs_err": abs(v - host.spec.analytic()), "seconds": s,
                     "subintervals_per_s": n / s})
    if a.integrand == "sin" and a.rule == "left" and not a.expr:
        pool = m.HostPool(a.threads)
        v, s = timed(lambda: m.host_riemann_mpi_parity(a.ranks, float(n), math.pi, pool), 1)
        rows.append({"side": "reference-program", "what": f"riemann.cpp as mpirun -np {a.ranks} "
                     f"runs it ({a.ranks - 1} workers on threads, scalar libm sin)", "value": v,
                     "abs_err": abs(v - 2.0), "seconds": s, "subintervals_per_s": n / s})
    if m.device_count() > 0 and a.expr:
        ei = m.ExprIntegrator(a.expr, 0)
        rl = getattr(m.Rule, a.rule)
        v = ei.integrate(lo, hi, n, rl, 0, n)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.06:  # clock settle
            ei.time(lo, hi, n, rl, 0, n, 4)
        s = ei.time(lo, hi, n, rl, 0, n, a.steps) * 1e-3
        rows.append({"side": "gpu", "what": f"{a.expr} compiled with hipRTC for gfx950",
                     "value": v, "seconds": s, "subintervals_per_s": n / s})
    elif m.device_count() > 0:
        gpu = Integrator(a.integrand, n=n, rule=a.rule)
        gpu.plan.prepare_steps(a.steps)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.06:  # clock settle, as bench.py (--settle-ms)
            gpu.run_steps(a.steps)
        t = gpu.run_steps(a.steps)
        v = gpu.plan.host_result(gpu.plan.host_index_of(a.steps - 1, True))
        s = t["device_ms"] * 1e-3 / a.steps
        rows.append({"side": "gpu", "what": f"MI355X HIP kernels, hipGraph batches of {a.steps}",
                     "value": v, "abs_err": abs(v - gpu.spec.analytic()), "seconds": s,
                     "subintervals_per_s": n / s})
    else:
        rows.append({"side": "gpu", "skipped": "no HIP device visible"})
    rate = {r["side"]: r.get("subintervals_per_s") for r in rows}
    for r in rows:
        print(json.dumps(r))
    if rate.get("gpu") and rate.get("host"):
        print(json.dumps({"speedup_gpu_vs_host": rate["gpu"] / rate["host"],
                          "speedup_gpu_vs_reference_program":
                          rate["gpu"] / rate["reference-program"]
                          if rate.get("reference-program") else None}))
    return 0


def cmd_integrate(a) -> int:
    from . import Integrator

    if a.expr:  # any f(x): compiled at run time with hipRTC (ops.kernels.riemann_expr)
        from .ops import kernels

        lo = 0.0 if a.a is None else a.a
        hi = 1.0 if a.b is None else a.b
        v = kernels.riemann_expr(a.expr, lo, hi, int(a.n), rule=a.rule)
        rec = {"expr": a.expr, "a": lo, "b": hi, "n": int(a.n), "rule": a.rule, "value": v}
        if a.analytic is not None:
            rec.update(analytic=a.analytic, abs_err=abs(v - a.analytic))
        print(json.dumps(rec))
        return 0

    ctx = _ctx()
    r = Integrator(a.integrand, n=int(a.n), rule=a.rule, dtype=a.dtype, div=a.div, ctx=ctx,
                   backend=a.backend).run()
    if ctx.is_root:
        print(json.dumps(r.as_dict()))
    ctx.destroy()
    return 0


def cmd_table2d(a) -> int:
    """BASELINE #5: the separable field v(x) v(y) over [0, 1800]^2 on a grid x grid midpoint
    grid, bilinear interpolation of the 1801^2 outer-product table; ranks split the rows."""
    from ._native import native

    ctx = _ctx("gloo" if a.backend == "cpu" else None)  # cpu: host tensors, host collective
    m = native()
    want = m.table2d_oracle(a.grid)
    rec = {"program": "table2d", "grid": a.grid, "gpus": ctx.world, "backend": a.backend}
    if a.backend == "cpu":
        import torch

        from .ops.kernels import table2d_reference
        from .utils import fixtures

        from .parallel.decomposition import rank_slice

        v = torch.as_tensor(fixtures.profile_table(), dtype=torch.float64)
        b, c = rank_slice(a.grid, ctx.rank, ctx.world)  # this rank's sample rows
        part = table2d_reference(torch.outer(v, v), 1800.0, 1800.0, a.grid, a.grid, b, b + c)
        rec["result"] = float(ctx.all_reduce_sum(torch.tensor([part], dtype=torch.float64))[0])
    else:
        from .parallel.dist import native_comm

        comm = native_comm(ctx) if ctx.world > 1 else None
        plan = m.Table2DPlan(a.grid, 1800.0, ctx.device, comm)
        rec["result"] = plan.run()
        rec["ms_per_integration"] = plan.time(a.iters, True)
        rec["samples_per_s"] = a.grid * a.grid / (rec["ms_per_integration"] * 1e-3)
    rec["midpoint_oracle"] = want
    rec["rel_err_vs_oracle"] = abs(rec["result"] - want) / want
    if ctx.is_root:
        print(json.dumps(rec))
    ctx.destroy()
    return 0


def cmd_oracle(a) -> int:
    from ._native import native

    m = native()
    o = m.oracle
    rows = {
        "profile_exact_integral": o.profile_exact_integral(),
        "cintegrate_sp32_sm2": o.cintegrate_parity(32, 2),
        "cintegrate_sp30_sm2": o.cintegrate_parity(30, 2),
        "cintegrate_sp32_sm3": o.cintegrate_parity(32, 3),
        "trainscan_p1": o.trainscan_parity(1)[0],
        "trainscan_p7": o.trainscan_parity(7)[0],
        "trainscan_p16": o.trainscan_parity(16)[0],
        "riemann_np8_n1e6": o.riemann_mpi_parity(8, 1e6),
        "train_analytic_1800": o.train_distance(1800.0),
        "pi4_left_n1e6_err": o.riemann_serial(m.Integrand.pi4, 0, 1, 10**6, m.Rule.left) - math.pi,
    }
    print(json.dumps(rows, indent=1))
    return 0


def cmd_info(a) -> int:
    from . import __version__
    from ._native import extension_path, native

    m = native()
    n = m.device_count()
    print(f"cuda_v_mpi_amd {__version__}  extension {extension_path()}")
    for d in range(n):
        print(" ", m.device_info(d))
    if n == 0:
        print("  no HIP device visible")
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="python -m cuda_v_mpi_amd", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)

    def common(sp, integrand="sin"):
        sp.add_argument("--integrand", default=integrand)
        sp.add_argument("--n", type=float, default=1e9)
        sp.add_argument("--rule", default="left", choices=["left", "mid", "right"])
        sp.add_argument("--dtype", default="fp64", choices=["fp64", "fp32", "fp32acc"])
        sp.add_argument("--div", default="series_exact", choices=["series", "ieee", "series_direct", "series_exact"])
        sp.add_argument("--block", type=int, default=256, choices=[64, 128, 256, 512, 1024],
                        help="threads per workgroup (the reference's SP)")
        sp.add_argument("--backend", default="hip", choices=["hip", "host", "cpu"])
        sp.add_argument("--json", action="store_true")

    common(sub.add_parser("riemann"))
    c = sub.add_parser("cintegrate")
    c.add_argument("--parity", action="store_true")
    c.add_argument("--sp", type=int, default=32)
    c.add_argument("--sm", type=int, default=2)
    c.add_argument("--backend", default="hip", choices=["hip", "host", "cpu"])
    c.add_argument("--json", action="store_true")
    t = sub.add_parser("trainscan")
    t.add_argument("--parity", action="store_true")
    t.add_argument("--algo", default="fused", choices=["fused", "onepass", "lookback"])
    t.add_argument("--json", action="store_true")
    ig = sub.add_parser("integrate")
    common(ig, integrand="pi4")
    ig.add_argument("--expr", default="", help="any f(x) as one C++ expression over x (hipRTC)")
    ig.add_argument("--a", type=float, default=None)
    ig.add_argument("--b", type=float, default=None)
    ig.add_argument("--analytic", type=float, default=None)
    t2 = sub.add_parser("table2d")
    t2.add_argument("--grid", type=int, default=4096)
    t2.add_argument("--iters", type=int, default=100)
    t2.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    sub.add_parser("oracle")
    sub.add_parser("info")
    cp = sub.add_parser("compare")
    cp.add_argument("--integrand", default="sin")
    cp.add_argument("--n", type=float, default=1e9)
    cp.add_argument("--rule", default="left", choices=["left", "mid", "right"])
    cp.add_argument("--threads", type=int, default=0)
    cp.add_argument("--ranks", type=int, default=8, help="reference program: mpirun -np P")
    cp.add_argument("--reps", type=int, default=3)
    cp.add_argument("--steps", type=int, default=48)
    cp.add_argument("--expr", default="", help="any f(x) as one C++ expression over x")
    cp.add_argument("--a", type=float, default=None)
    cp.add_argument("--b", type=float, default=None)
    sc = sub.add_parser("scale")
    sc.add_argument("--gpus", default="1,2,4,8")
    sc.add_argument("--steps", type=int, default=200)
    sc.add_argument("--warmup", type=int, default=10)
    sc.add_argument("--no-comm", action="store_true")
    sc.add_argument("--jsonl", default="")
    sc.add_argument("--md", default="")
    a = p.parse_args(argv)
    if a.cmd == "scale":
        from .parallel import scaling

        return scaling.main(["--gpus", a.gpus, "--steps", str(a.steps), "--warmup",
                             str(a.warmup)] + (["--no-comm"] if a.no_comm else []) +
                            (["--jsonl", a.jsonl] if a.jsonl else []) +
                            (["--md", a.md] if a.md else []))
    return {"riemann": cmd_riemann, "cintegrate": cmd_cintegrate, "trainscan": cmd_trainscan,
            "integrate": cmd_integrate, "table2d": cmd_table2d, "oracle": cmd_oracle,
            "info": cmd_info, "compare": cmd_compare}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
