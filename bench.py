#!/usr/bin/env python3
"""Headline benchmark: Riemann subintervals/s of 4/(1+x^2) on [0,1], N=1e9 fp64.

Metric and config come from BASELINE.json ("Riemann subintervals/sec at N=1e9 fp64; |error|
vs analytic pi"). One step = one complete integration of N = 1e9 samples IN TOTAL, split over
the G GPUs as the reference splits its fixed STEPS over its workers (riemann.cpp:10,71-73:
strong scaling, so the record at every G is the metric's own config): gfx950 kernel (every
sample evaluated, fp64) -> in-kernel DPP/LDS reduction -> RCCL all-reduce of the per-GPU
partial over xGMI -> D2H into pinned memory. Steps run in batches of --slots (48) steps plus
one remainder-sized batch; a batch is ONE persistent multi-step launch of all its steps and a
closing kernel, enqueued directly (--graph-batches: as a hipGraph replay, captured before the
warmup; measured slower, profiles/r5/graph_vs_direct.md); with >1 GPU each batch ends in ONE all-reduce of its
step results (bucketed: every step still gets its own global sum; --no-bucket = one 8-byte
all-reduce per step, overlapped on a side stream).

Launch (the reference's `mpirun -np P ./riemann`, riemann.cpp:62-86: one command, P ranks,
one gathered result):

    python bench.py                          # 1 GPU, in this process
    python bench.py --gpus 8                 # spawns 8 rank processes (one per GPU)
    torchrun --nproc-per-node 8 bench.py --gpus 8     # the same ranks under torchrun

With --gpus N > 1 and no torchrun environment, this process only spawns N children with
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT set and relays their exit status; it
never imports torch or touches the GPU itself. Every child runs the torchrun path.

Warmup: the W warmup steps, then untimed repeats of the timed K-step pattern for at least
--settle-ms (60) so the timed region starts at steady clocks (from idle the GPU ramps from
~90 to 76.8 us per step over ~25 ms), then one more K-step pattern on its own (launch, sync):
the first launch call after a sync that drained a run of queued launches holds the host
6-8 us longer than the next ones, with the GPU idle behind it (tools/share_duty_probe.py,
profiles/r6/batch_tail.md). The JSON line reports all of these as "warmup_settle_steps".

Scaling: the headline is strong (N = 1e9 in total; --scaling weak makes --samples a per-GPU
count instead). The results of the last batch of timed steps (every rank holds the global
sums) are checked on the host against the rule's closed-form truncation error. After the timed
region (outside it) the same ranks also measure, each with its own graphs, timing and
pass/fail ("verified"): the weak-scaling form, 1e9 samples PER GPU (N = 1e9 x G,
"weak_1e9_per_gpu"); the same config with IEEE division per sample ("ieee_div"); the headline
division's per-point error against IEEE division and against the true value on two 64 K-sample
windows ("per_point"); and the other BASELINE configs: #1, the serial CPU sum at N = 1e6 on one host thread
("baseline1_serial_cpu_1e6"); #3, N = 1e10 in total strong-scaled over the same GPUs
("baseline3_strong_1e10"); #4, the same integral through the packed-fp32 path
("baseline4_fp32", tile values folded in fp64, and "baseline4_fp32_accum32", fp32 accumulation
to the workgroup partial); #5, the 4096^2 2-D velocity field with its rows split over the same
GPUs ("baseline5_table2d_4096") — and the same integral on the node's host cores (the native
host engine, the reference's own CPU/MPI side: "host_engine"). Also: one integration per call,
launch to pinned result, the reference's own timing unit ("single_shot_1e9"); the headline
config with the faster g = 1/2 + e series fold (up to 5 ulp per point: "series_div"); and the
reference's own integrands through the same batches ("integrand_sin", "integrand_train",
"integrand_table", "integrand_poly"). The record's "verified" is the AND of the headline's,
every extra's and the RCCL transport check ("transport_verified": ranks of one node on distinct
GPUs must be SEEN to meet over xGMI peer-to-peer; a network transport or no transport evidence
at all fails it); the exit status follows the headline's.

One RCCL communicator per rank: with --comm native (default) the torch process group is gloo
and carries only the control plane (barriers, the settle-count MAX, the per-rank times); the
native communicator is shared by every plan of the run. The record says which
("control_plane", "torch_nccl_groups").
"""
from __future__ import annotations

import argparse
import json
import math
import os
import signal
import socket
import subprocess
import sys
import time

# Reference-algorithm number for the same metric/config, measured by the survey on a CPU
# (the reference's left-Riemann loop, riemann.cpp:29-44, applied to 4/(1+x^2),
# N=1e9, 8 Xeon workers, -O2): 0.203 s -> 4.94e9 subintervals/s, |err| 1.000e-9. The
# reference publishes no numbers of its own (BASELINE.json "published": {}).
BASELINE_SUBINT_PER_S = 4.94e9
BASELINE_SOURCE = ("CPU reimplementation of the reference algorithm (8 Xeon cores, -O2, "
                   "BASELINE.md); the reference publishes no numbers")


def parse(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--settle-ms", type=float, default=60.0,
                   help="after the W warmup steps, repeat the timed K-step pattern (untimed) "
                        "for at least this long so the timed steps run at steady clocks (0 = off)")
    # (--n is a prefix of torchrun's own --nnodes/--nproc-per-node: use --samples under torchrun)
    p.add_argument("--no-rearm-batch", action="store_true",
                   help="A-B: no untimed K-step pattern on its own between the settle and the "
                        "timed region")
    p.add_argument("--samples", "--n", dest="n", type=float, default=1e9,
                   help="samples in total (strong, the default: the metric's N = 1e9 split "
                        "over the GPUs) or per GPU (--scaling weak)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                   help="strong: N fixed in total (riemann.cpp:10,71-73); weak: N per GPU")
    p.add_argument("--integrand", default="pi4")
    p.add_argument("--rule", default="left", choices=["left", "mid", "right"])
    p.add_argument("--dtype", default="fp64", choices=["fp64", "fp32", "fp32acc"],
                   help="fp32acc: fp32 samples AND fp32 accumulation to the workgroup partial "
                        "(pi4 only; fp32 folds tile values into fp64)")
    p.add_argument("--div", default="series_exact", choices=["series", "ieee", "series_direct", "series_exact"])
    p.add_argument("--comm", default="native", choices=["native", "torch"],
                   help="native: C++ RCCL communicator captured in the step graph; "
                        "torch: torch.distributed all_reduce of each step's partial")
    p.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                   help="torch process-group backend. Default: gloo with --comm native (the "
                        "group carries only the control plane; the rank's one RCCL "
                        "communicator is the native one), nccl with --comm torch, gloo with "
                        "--device cpu")
    p.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                   help="cpu: torch fp64 evaluation + gloo (launcher / decomposition tests "
                        "on a GPU-less box; not a performance configuration)")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--graph-batches", action="store_true",
                   help="replay multi-step batches as hipGraphs (default: launch their two "
                        "kernels directly, measured faster; profiles/r5/graph_vs_direct.md)")
    p.add_argument("--no-pipeline", action="store_true")
    p.add_argument("--unfused", action="store_true", help="partials + finalize (2 launches)")
    p.add_argument("--grid", type=int, default=0, help="workgroups (0 = auto; the reference's SM)")
    p.add_argument("--block", type=int, default=256, choices=[64, 128, 256, 512, 1024],
                   help="threads per workgroup (the reference's SP)")
    p.add_argument("--slots", type=int, default=48,
                   help="steps per captured graph batch (= steps per bucketed all-reduce)")
    p.add_argument("--step-streams", type=int, default=0,
                   help="streams a chained graph batch deals its steps over (0 = auto: 4 below "
                        "6e8 samples per GPU per step, else 1)")
    p.add_argument("--no-multistep", action="store_true",
                   help="graph batches as one kernel launch per step (chained) instead of one "
                        "persistent launch for the whole batch")
    p.add_argument("--no-bucket", action="store_true",
                   help="one all-reduce per step instead of one per graph batch of steps")
    p.add_argument("--force-collective", action="store_true",
                   help="run the RCCL all-reduce stage even on 1 GPU (tests the multi-GPU graph)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the post-timing extras (IEEE run, per-point ulp, BASELINE #1, #3, #4, #5, "
                        "host engine)")
    p.add_argument("--sweep-gpus", default="",
                   help="e.g. 1,2,4,8: run the scaling sweep (cuda_v_mpi_amd/parallel/scaling.py) "
                        "over these GPU counts instead of one benchmark")
    p.add_argument("--no-diag", action="store_true",
                   help="skip the untimed diagnostic batch and communicator probes that a "
                        "multi-rank run records after its timed region (diagnostic_batch)")
    p.add_argument("--diag-allgather-mb", type=float, default=144.0,
                   help="total size of the diagnostic allgather (the reference's 144 MB "
                        "table, 4main.c:157)")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--jsonl", default="", help="also append the JSON line to this file")
    return p.parse_args(argv)


# ------------------------------------------------------------------ launcher (no GPU here)
def rendezvous_port(offsets=(0, 17, 19)) -> int:
    """A MASTER_PORT P with P + o free for every offset o (the native CLIs add 17 and 19), below
    the kernel's ephemeral range: a port from bind(0) lies inside it, where a rank retrying its
    connect() can be handed it as a local port and self-connect (csrc/include/miint/net.hpp)."""
    import random

    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            low = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        low = 32768
    hi = low - max(offsets)
    lo = 20000 if hi > 21000 else 1024

    def free(port: int) -> bool:
        with socket.socket() as s:
            try:
                s.bind(("", port))
                return True
            except OSError:
                return False

    for _ in range(64):
        p = random.randint(lo, hi - 1)
        if all(free(p + o) for o in offsets):
            return p
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Start n rank processes of this script and wait for them (mpirun -np n analogue).

    Runs before anything imports torch or the native extension, so this process never
    initialises HIP (a GPU-initialised parent may not fork/exec on the pool). The first rank
    that fails ends the others; the exit status is the first non-zero one.
    """
    port = rendezvous_port()
    base = dict(os.environ)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), MIINT_BENCH_LAUNCHER="spawn",
                MIINT_BENCH_PARENT_TORCH="1" if "torch" in sys.modules else "0")
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=env))

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    def on_signal(signum, _frame):
        stop_all()
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    linger_until = None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            # a rank that exited with a status (not a signal) may be one of several ending the
            # same agreed failure (a verification every rank computes alike): give the others
            # 2 s to finish, so rank 0's record is printed rather than cut off
            if bad and rc == 0 and linger_until is None and bad[0] > 0:
                linger_until = time.time() + 2.0
            if bad and rc == 0 and (bad[0] < 0 or time.time() >= linger_until
                                    or all(c is not None for c in codes)):
                rc = bad[0]
                print(f"bench.py: a rank exited with {rc}; stopping the others", file=sys.stderr)
                stop_all()
                t_end = time.time() + 15
                while any(p.poll() is None for p in procs) and time.time() < t_end:
                    time.sleep(0.1)
                stop_all(signal.SIGKILL)
            if all(c is not None for c in (p.poll() for p in procs)):
                break
            time.sleep(0.05)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc


# ------------------------------------------------------------------ per-rank benchmark
def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.sweep_gpus:
        from cuda_v_mpi_amd.parallel import scaling

        return scaling.main(["--gpus", args.sweep_gpus, "--steps", str(args.steps),
                             "--warmup", str(args.warmup)] +
                            (["--jsonl", args.jsonl] if args.jsonl else []))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1 and "RANK" not in os.environ:
        return spawn_ranks(args.gpus, argv)
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    launcher = os.environ.get("MIINT_BENCH_LAUNCHER",
                              "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or world_env > 1
                              else "single")

    import torch

    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.parallel import dist as mdist

    cpu = args.device == "cpu"
    if not cpu:
        # RCCL's INIT log into a per-process file before anything initialises RCCL (the
        # native communicator, or torch's with --comm torch): the record names the transport
        from cuda_v_mpi_amd import native as _native_mod

        _native_mod().capture_rccl_log()
    backend_auto = args.backend is None
    if backend_auto:
        args.backend = mdist.control_backend(args.comm, args.device)
    if cpu and args.backend != "gloo" and world_env > 1:
        print("bench.py: --device cpu needs --backend gloo", file=sys.stderr)
        return 2
    ctx = mdist.init(backend=args.backend, force=False)
    world = ctx.world
    for k, want in (("RANK", ctx.rank), ("LOCAL_RANK", ctx.local_rank), ("WORLD_SIZE", world)):
        assert int(os.environ.get(k, str(want))) == want, (k, os.environ.get(k), want)
    n_per = int(args.n)
    n_total = n_per * world if args.scaling == "weak" else n_per
    dev = "cpu" if (cpu or ctx.host_collectives) else "cuda"  # control-plane tensors

    def sync_dev():
        if not cpu:
            torch.cuda.synchronize()

    def make_integ(comm):
        return Integrator(args.integrand, n=n_total, rule=args.rule, dtype=args.dtype,
                          div=args.div, backend="cpu" if cpu else "hip", ctx=ctx, comm=comm,
                          fused=not args.unfused, grid=args.grid, slots=args.slots,
                          force_collective=args.force_collective, bucket=not args.no_bucket,
                          step_streams=args.step_streams, block=args.block,
                          multistep=not args.no_multistep)

    # A native RCCL communicator that fails to come up on every rank (the failure is agreed
    # over the torch process group, so all ranks switch together) falls back to the
    # torch.distributed step path instead of ending the run without a record.
    comm_fallback = None
    try:
        integ, init_error = make_integ(args.comm), None
    except Exception as e:  # noqa: BLE001
        integ, init_error = None, e
    if world > 1 and not cpu and args.comm == "native":
        flag = torch.tensor([0.0 if init_error is None else 1.0], dtype=torch.float64, device=dev)
        ctx.all_reduce_max(flag)
        if flag.item() > 0:
            comm_fallback = (f"{type(init_error).__name__}: {init_error}" if init_error
                             else "a peer rank failed to create the native communicator")
            print(f"bench.py: native RCCL communicator failed ({comm_fallback}); "
                  "falling back to --comm torch", file=sys.stderr)
            args.comm = "torch"
            integ, init_error = make_integ("torch"), None
    if init_error is not None:
        raise init_error
    use_torch = args.comm == "torch" and world > 1 and not cpu
    plan = integ.plan
    graphs = not args.no_graph and not use_torch and not cpu
    # A multi-step plan's batch is two launches (the persistent launch of all its steps and
    # the closing kernel; then the all-reduce and the copy on several GPUs). Enqueued
    # directly they ran ~1 % (one GPU) and 2-4 % (the 1/8 share of an 8-GPU step) faster than
    # the same nodes as a graph replay (profiles/r5/graph_vs_direct.md): a hipGraphLaunch
    # costs more than two kernel launches. --graph-batches replays them anyway.
    direct_batches = bool(graphs and plan is not None and plan.multistep
                          and not args.graph_batches)
    if direct_batches:
        graphs = False
    ran_plan = plan is not None and not use_torch and not cpu  # the native plan ran the steps
    pipeline = not args.no_pipeline and (world > 1 or args.force_collective)

    if cpu:  # torch fp64 evaluation of the rank slice + gloo all_reduce per step
        cpu_vals: list[float] = []

        def launch(k):
            for _ in range(k):
                cpu_vals.append(integ.run().value)
        finish = lambda: None  # noqa: E731
        result = lambda k: cpu_vals[len(cpu_vals) - args.steps + k]  # noqa: E731
    elif use_torch:  # kernels on the torch stream + torch.distributed all_reduce per step
        from cuda_v_mpi_amd.parallel.torch_steps import TorchStepper

        # an auto-chosen gloo control plane gets an RCCL group for the device collectives; an
        # explicit --backend gloo (ranks sharing one GPU) keeps gloo on CUDA tensors
        group = ctx.nccl_group() if (backend_auto and ctx.host_collectives) else None
        stepper = TorchStepper(integ.spec, n_total, ctx, rule=args.rule, dtype=args.dtype,
                               div=args.div, grid=args.grid or None, group=group)
        launch, finish, result = stepper.launch_steps, stepper.sync, stepper.result
    else:
        if graphs:  # capture every graph the timed pattern replays, before anything is timed
            plan.prepare_steps(args.steps)
            if not plan.graphs_ready:
                print(f"bench.py: hipGraph capture failed ({plan.graph_error}); "
                      "running with direct stream enqueue", file=sys.stderr)
                graphs = False
        launch = lambda k: plan.launch_steps(k, pipeline, graphs)  # noqa: E731
        finish = plan.sync
        result = lambda k: plan.host_result(plan.host_index_of(k, graphs))  # noqa: E731

    # ---- warmup (RCCL channel setup, code-object load, first replays)
    launch(max(1, args.warmup))
    finish()
    # ---- clock settle: from idle the MI355X needs ~25 ms of continuous work before its
    # per-step time is steady (90 -> 76.8 us per step; profiles/r1/clock_ramp.jsonl). The
    # settle phase repeats exactly the timed K-step pattern (same graphs, same remainder
    # batch), for at least --settle-ms; the repeat count is calibrated once and agreed across
    # ranks (MAX) so every rank runs the same collectives.
    settle_steps = 0
    if args.settle_ms > 0 and not cpu:
        t_c = time.perf_counter()
        launch(args.steps)
        finish()
        per_call = time.perf_counter() - t_c
        want = torch.tensor([math.ceil(args.settle_ms * 1e-3 / max(per_call, 1e-7))],
                            dtype=torch.float64, device=dev)
        ctx.all_reduce_max(want)
        calls = int(want.item())
        for _ in range(calls):
            launch(args.steps)
        finish()
        settle_steps = (1 + calls) * args.steps
    rearm = not cpu and not args.no_rearm_batch
    # the native plan on several GPUs has a device barrier of its own (below); there the host
    # barrier comes BEFORE the re-arm batch, so the GPU does not sit idle through it right
    # before the clock: a batch that follows >= 100 us of idle GPU runs 4-7 us slower at the
    # 1/8 share (share_duty_probe.py --idle-us), and a gloo barrier of 8 local ranks takes
    # ~100-300 us (profiles/r6/batch_tail.md)
    device_barrier = ran_plan and world > 1
    if rearm:
        if device_barrier:
            ctx.barrier()
        # the timed pattern once more, launched and synced on its own: the first launch call
        # after the sync that drained the queued settle (or warmup) launches costs the host
        # 6-8 us more than a launch after a synced one, while the GPU waits for it; the
        # timed region's launch should be the steady one (tools/share_duty_probe.py: at the
        # 1/8 share 210.4 -> 202.3 us per 20-step batch, profiles/r6/batch_tail.md)
        launch(args.steps)
        finish()
        settle_steps += args.steps

    # ---- timed region: barrier + device sync on both sides, K steps in between
    g0 = plan.graph_launches if plan is not None else 0
    d0 = plan.direct_steps if plan is not None else 0
    if not (rearm and device_barrier):
        ctx.barrier()
    if plan is not None and not cpu:
        # then a device barrier through the rank's RCCL communicator (an 8-byte all-reduce on
        # the compute stream, polled): ranks leave a host barrier (or the re-arm batch's
        # all-reduce) up to tens of us apart,
        # and the early ones would count that skew as step time inside the batch's
        # all-reduce; an all-reduce completes on every rank within ~us (no-op on one GPU)
        plan.barrier()
    sync_dev()
    t0 = time.perf_counter()
    launch(args.steps)
    finish()
    sync_dev()
    t1 = time.perf_counter()
    ctx.barrier()
    elapsed = t1 - t0
    graph_replays = (plan.graph_launches - g0) if plan is not None else 0
    direct_timed = (plan.direct_steps - d0) if plan is not None else args.steps

    per_rank_ms = ctx.all_gather_scalars(elapsed / args.steps * 1e3, device=dev)
    elapsed_max = max(per_rank_ms) * args.steps * 1e-3

    # ---- verify the results of the last steps (every rank holds the global value)
    analytic = integ.spec.analytic()
    slots = plan.slots if plan is not None else args.slots
    last = range(max(0, args.steps - min(args.steps, slots)), args.steps)
    vals = [result(k) for k in last]
    errs = [abs(v - analytic) for v in vals]
    abs_err = max(errs)
    ok = all(math.isfinite(v) for v in vals) and all(
        result_ok(args.integrand, args.rule, args.dtype, n_total, e, integ.spec) for e in errs)

    ms_per_step = elapsed_max / args.steps * 1e3
    value = n_total * args.steps / elapsed_max

    # ---- outside the timed region: transport facts and the extras
    comm = getattr(integ, "_comm", None)
    rccl_world = comm.transport_world if comm is not None else None
    rccl_version = None
    transport = {}
    if not cpu:
        from cuda_v_mpi_amd import native

        rccl_version = native().Comm.version()
        if world > 1:
            transport = native().rccl_transport()
    native_rccl = int(comm is not None and getattr(comm, "kind", "") == "rccl")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # ranks share GPUs: MIINT_OVERSUBSCRIBE, or simply more local ranks than devices (gloo
    # rehearsals on one GPU map rank r to device r % count)
    share = world > 1 and (mdist.ranks_share_devices() or
                           (not cpu and local_world > torch.cuda.device_count()))
    # the transport check applies only where RCCL carried the ranks' collectives
    transport_error = transport_check(world, share, transport,
                                      rccl=not cpu and bool(native_rccl or ctx.nccl_groups))
    native_comm_ok = comm_fallback is None
    if transport_error:
        print(f"bench.py: {transport_error}", file=sys.stderr)
    diag = None
    if world > 1 and not args.no_diag:
        # untimed, after the timed region: where a multi-GPU step's time went
        try:
            diag = batch_diagnostics(args, ctx, integ, plan, dev, cpu, use_torch, transport)
        except Exception as e:  # noqa: BLE001  (every rank runs the same probes)
            diag = {"error": f"{type(e).__name__}: {e}"}
            print(f"bench.py: diagnostics failed: {diag['error']}", file=sys.stderr)
    extras = {}
    extras_ok = True
    if not cpu and not use_torch and not args.no_extras:
        # The headline is already measured: a failure in an extra must not cost the record.
        # (Every rank runs the same extras, so an exception on one is one on all; the
        # collective sequence stays matched.)
        try:
            extras = run_extras(args, ctx, integ, n_total, pipeline, dev)
        except Exception as e:  # noqa: BLE001
            extras = {"extras_error": f"{type(e).__name__}: {e}"}
            print(f"bench.py: extras failed: {extras['extras_error']}", file=sys.stderr)
        # every extra carries its own pass/fail; the record's `verified` is the AND of all
        extras_ok = "extras_error" not in extras and all(
            v.get("verified", True) for v in extras.values() if isinstance(v, dict))

    if ctx.is_root:
        out = {
            # BASELINE.json's metric string, verbatim
            "metric": "Riemann subintervals/sec at N=1e9 fp64; |error| vs analytic \u03c0",
            "value": value,
            "unit": "subintervals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_settle_steps": settle_steps,
            # the untimed K-step pattern launched and synced on its own right before the clock
            "warmup_rearm_batch": rearm,
            # what stands right before the clock: the host barrier (control plane), the native
            # plan's RCCL device barrier, or the device barrier alone with the host barrier
            # moved before the re-arm batch
            "pre_clock_barrier": ("device" if (rearm and device_barrier) else
                                  "host+device" if (plan is not None and not cpu and world > 1
                                                    and ran_plan) else "host"),
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": value / BASELINE_SUBINT_PER_S,
            "baseline_source": BASELINE_SOURCE,
            "dtype": args.dtype,
            "data": "synthetic (analytic integrand 4/(1+x^2); no dataset)",
            "abs_err": abs_err,
            "result": vals[-1],
            "verified": record_verified(ok, extras_ok, transport_error, comm_fallback),
            "headline_verified": ok,
            "native_comm_verified": native_comm_ok,
            "extras_verified": extras_ok,
            "transport_verified": not transport_error,
            "transport_error": transport_error,
            "verify_rule": verify_rule(args.integrand, args.rule, args.dtype),
            "launcher": launcher,
            "parent_imported_torch": os.environ.get("MIINT_BENCH_PARENT_TORCH") == "1",
            "rccl_world": rccl_world,
            "rccl_version": rccl_version,
            # what RCCL's INIT log says rank 0's connections use (P2P/IPC over xGMI on one
            # node; NET/Socket when ranks share a GPU) and how many nodes it counted
            "rccl_transport": transport.get("transport") if transport else None,
            "rccl_nnodes": transport.get("nnodes") if transport else None,
            "rccl_connections": transport.get("connections") if transport else None,
            # one RCCL communicator per rank: the native one (data plane); the torch group is
            # the control plane (gloo unless --comm torch), torch RCCL groups counted here
            "control_plane": ctx.backend,
            "torch_nccl_groups": ctx.nccl_groups,
            "native_rccl_comms": native_rccl,
            # MIINT_OVERSUBSCRIBE: ranks share GPUs and RCCL runs over loopback sockets — a
            # correctness run of the multi-rank path, not a scaling number
            "ranks_share_gpus": share,
            "per_rank_ms": per_rank_ms,
            "per_rank_spread_ms": max(per_rank_ms) - min(per_rank_ms),
            "graph_replays_timed": graph_replays,
            "comm_fallback": comm_fallback,
            "direct_steps_timed": direct_timed,
            **({"diagnostic_batch": diag} if diag is not None else {}),
            **extras,
            "config": {
                "model": f"riemann_{args.integrand}_{args.dtype}",
                "integrand": "4/(1+x^2) on [0,1]" if args.integrand == "pi4" else args.integrand,
                "N": n_total,
                # rank 0's share (ranks differ by at most one sample when G does not divide N)
                "n_per_gpu": plan.count if plan is not None else n_total // world,
                "rule": args.rule,
                "division": str(plan.effective_div).split(".")[-1] if plan is not None else "ieee",
                "global_batch": n_total,
                "seq_len": 1,
                "parallelism": f"dp{world}",
                "comm": (args.comm if (world > 1 or args.force_collective) else "none"),
                # true only when the timed region ran as graph replays and nothing else
                "graphs": bool(graphs and graph_replays > 0 and direct_timed == 0),
                "graph_nodes": plan.graph_nodes if (graphs and plan is not None) else 0,
                "pipeline": pipeline,
                "bucketed_allreduce": bool(plan.bucketed) if plan is not None else False,
                # the bucketed all-reduce writes every rank's step values straight into
                # pinned host memory (no copy after it); multi-step batches closed inside the
                # persistent launch instead of by a closing kernel
                # (graph replays keep the device buffer + copy node: RiemannConfig)
                "allreduce_to_host": bool(plan is not None and plan.allreduce_to_host and
                                          not graphs),
                "close_in_launch": bool(plan.close_in_launch) if plan is not None else False,
                "fused_reduction": not args.unfused,
                "chained_batches": bool(ran_plan and plan.chained and (graphs or plan.multistep)),
                # a batch is ONE persistent launch of all its steps + a closing kernel
                "multistep": bool(ran_plan and plan.multistep),
                # how the timed batches were launched: a graph replay, a multi-step batch's
                # two kernels enqueued directly, or one launch per step
                "batch_launch": ("graph" if graphs else
                                 "direct" if ran_plan and plan.multistep else
                                 "per-step" if ran_plan else "none"),
                "step_streams": plan.step_streams(min(args.steps, plan.slots))
                if plan is not None else 1,
                "grid": plan.grid if plan is not None else 0,
                "block": plan.block if plan is not None else args.block,
                "device": args.device,
            },
        }
        print(json.dumps(out), flush=True)
        if args.jsonl:
            with open(args.jsonl, "a") as f:
                f.write(json.dumps(out) + "\n")
    ctx.destroy()
    return 0 if ok else 1


def _spread(vals: list[float]) -> dict:
    return {"max": max(vals), "min": min(vals), "per_rank": vals}


def rccl_init_lines(path: str | None, limit: int = 16) -> dict:
    """Channel and protocol facts from this rank's captured RCCL INIT log (NCCL_DEBUG_SUBSYS
    INIT,P2P,GRAPH: printed once per communicator): the distinct channel ids of the peer
    connections, and the lines naming channels, rings, trees or protocols (RCCL's LL cutoff
    warning among them). The per-call algorithm/protocol choice is a TUNING line RCCL prints
    for EVERY collective — a file write inside the timed region — so it is not captured."""
    import re

    if not path or not os.path.exists(path):
        return {"log": path, "channels": None, "lines": []}
    chans, lines = set(), []
    keep = re.compile(r"channels|nChannels|Pattern|Ring \d+|[Pp]roto|LL128|LL cutoff|Tree \d+")
    with open(path, errors="replace") as f:
        for ln in f:
            m = re.search(r"Channel (\d+)/\d+ :", ln)
            if m:
                chans.add(int(m.group(1)))
            elif keep.search(ln) and len(lines) < limit:
                lines.append(ln.split("NCCL INFO", 1)[-1].strip())
    return {"log": path, "channels": len(chans) or None, "lines": lines}


def comm_probes(ctx, comm, allgather_mb: float, cpu: bool) -> dict:
    """Latency of an 8-byte all-reduce and the bus bandwidth of an allgather of
    `allgather_mb` MB in total (each rank's 1/world share), on the run's own communicator:
    the native RCCL one (hipEvents on the torch stream), or, on the CPU path, the gloo group.
    busbw = total bytes x (world - 1) / world / time (the ring's per-link traffic)."""
    import statistics

    import torch
    import torch.distributed as tdist

    world = ctx.world
    per = max(1, int(allgather_mb * 1e6 / 8) // world)
    out: dict = {"allgather_bytes": per * world * 8, "world": world}
    if cpu or comm is None:
        x = torch.zeros(1, dtype=torch.float64)
        for _ in range(5):
            tdist.all_reduce(x)
        lat = []
        for _ in range(20):
            t = time.perf_counter()
            tdist.all_reduce(x)
            lat.append((time.perf_counter() - t) * 1e6)
        send = torch.zeros(per, dtype=torch.float64)
        recv = [torch.empty(per, dtype=torch.float64) for _ in range(world)]
        tdist.all_gather(recv, send)
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            tdist.all_gather(recv, send)
            ts.append(time.perf_counter() - t)
        out.update(transport="gloo", allreduce_8b_us=statistics.median(lat))
        t_ag = min(ts)
    else:
        s = torch.cuda.current_stream()
        x = torch.zeros(1, dtype=torch.float64, device="cuda")
        for _ in range(20):
            comm.allreduce_sum(x.data_ptr(), x.data_ptr(), 1, s.cuda_stream)
        lat = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(50):
                comm.allreduce_sum(x.data_ptr(), x.data_ptr(), 1, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            lat.append(e0.elapsed_time(e1) * 1e3 / 50)
        send = torch.zeros(per, dtype=torch.float64, device="cuda")
        recv = torch.empty(per * world, dtype=torch.float64, device="cuda")
        for _ in range(2):
            comm.allgather(send.data_ptr(), recv.data_ptr(), per, s.cuda_stream)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            comm.allgather(send.data_ptr(), recv.data_ptr(), per, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        out.update(transport=getattr(comm, "kind", "native"),
                   allreduce_8b_us=statistics.median(lat))
        t_ag = min(ts)
        del send, recv
    # the slowest rank's numbers
    m = torch.tensor([out["allreduce_8b_us"], t_ag], dtype=torch.float64,
                     device="cpu" if (cpu or ctx.host_collectives) else "cuda")
    ctx.all_reduce_max(m)
    total = per * world * 8
    out.update(allreduce_8b_us=float(m[0]), allgather_s=float(m[1]),
               allgather_algbw_gbs=total / float(m[1]) / 1e9,
               allgather_busbw_gbs=total * (world - 1) / world / float(m[1]) / 1e9)
    return out


def batch_diagnostics(args, ctx, integ, plan, dev, cpu: bool, use_torch: bool,
                      transport: dict) -> dict:
    """VERDICT r5 Next #2: one untimed batch after the timed region, taken apart on every
    rank — compute (the batch's kernels), tail (closing kernel + all-reduce + copy to pinned
    memory), the kernel boundaries the stage events stood in for (device - compute - tail) and
    the host's part (wall - device) — with the max and min over ranks; then the
    communicator's 8-byte all-reduce latency and allgather bus bandwidth, and RCCL's channel
    and protocol lines from rank 0's INIT log. These say where a multi-GPU step's time went
    (the reference's reduce / barrier / broadcast costs, 4main.c:134-157)."""
    import torch

    steps = min(args.steps, plan.slots if plan is not None else args.slots)
    keys = ("compute_us", "close_us", "allreduce_us", "copy_us", "tail_us", "boundary_us",
            "device_us", "wall_us", "marker_us")
    if cpu:  # as the timed CPU steps run: per step the torch fp64 evaluation of the rank's
        # slice, then its gloo all-reduce (which also waits for the slowest rank)
        comp = red = 0.0
        t_start = time.perf_counter()
        for _ in range(steps):
            t0 = time.perf_counter()
            v = torch.tensor([integ._cpu_local()], dtype=torch.float64)
            t1 = time.perf_counter()
            ctx.all_reduce_sum(v)
            t2 = time.perf_counter()
            comp, red = comp + (t1 - t0), red + (t2 - t1)
        wall = time.perf_counter() - t_start
        d = {"steps": steps, "compute_us": comp * 1e6, "close_us": 0.0,
             "allreduce_us": red * 1e6, "copy_us": 0.0, "tail_us": red * 1e6, "boundary_us": 0.0,
             "device_us": (comp + red) * 1e6, "wall_us": wall * 1e6, "marker_us": 0.0,
             "path": "cpu"}
    elif use_torch or plan is None:
        d = {"steps": steps, "path": "torch", **{k: None for k in keys}}
    else:
        d = dict(plan.diagnose_batch(steps), path="native",
                 close_in_launch=bool(plan.close_in_launch),
                 allreduce_to_host=bool(plan.allreduce_to_host))
    out: dict = {"steps": d["steps"], "path": d["path"]}
    for k in keys:
        if d.get(k) is None:
            out[k] = None
            continue
        out[k] = _spread(ctx.all_gather_scalars(float(d[k]), device=dev))
    out["host_us"] = (None if d.get("wall_us") is None else
                      _spread(ctx.all_gather_scalars(float(d["wall_us"] - d["device_us"]),
                                                     device=dev)))
    for k in ("close_in_launch", "allreduce_to_host"):
        if k in d:
            out[k] = d[k]
    if not use_torch:
        out["comm"] = comm_probes(ctx, getattr(integ, "_comm", None), args.diag_allgather_mb,
                                  cpu)
    if not cpu:
        out["rccl_init"] = rccl_init_lines((transport or {}).get("log"))
    return out


def record_verified(headline_ok: bool, extras_ok: bool, transport_error: str | None,
                    comm_fallback: str | None) -> bool:
    """The record's `verified`: the headline's check AND every extra's AND the transport check
    AND the native communicator having carried the run. A native-communicator failure that the
    run survived on the torch.distributed data plane (comm_fallback) still fails it: the
    record stands for the native RCCL path, and a fallback there would otherwise turn a
    native-comm bug into a passing record on another code path (native_comm_verified)."""
    return bool(headline_ok and extras_ok and not transport_error and comm_fallback is None)


def transport_check(world: int, share: bool, transport: dict, rccl: bool = True) -> str | None:
    """None, or why the multi-GPU record cannot stand: ranks of ONE node on distinct GPUs must
    be seen to meet over xGMI peer-to-peer, not a network transport (a silent fallback — P2P
    disabled, a leaked NCCL_HOSTID splitting the node into W "hosts" — would corrupt the scaling
    curve). Fail-closed: no transport evidence at all (RCCL's INIT log missing or without a
    single peer connection) fails too, since it cannot tell xGMI from sockets. Ranks sharing a
    GPU (MIINT_OVERSUBSCRIBE) legitimately use sockets; gloo-only runs (rccl=False) have no
    RCCL transport to check."""
    if world <= 1 or share or not rccl:
        return None
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if local != world:  # a multi-node job: NET between nodes is expected
        return None
    if not transport or not transport.get("transport"):
        where = (transport or {}).get("log") or "no RCCL log captured"
        return (f"RCCL transport unknown between {world} ranks on distinct local GPUs (no peer "
                f"connection in {where}): P2P over xGMI cannot be confirmed")
    if transport.get("uses_net") or not all(t.startswith("P2P")
                                            for t in transport["transport"].split("+")):
        # a network transport, or shared host memory (SHM: P2P disabled) — not xGMI
        return (f"RCCL transport is {transport['transport']} (nNodes {transport.get('nnodes')}) "
                f"between {world} ranks on distinct local GPUs: expected P2P over xGMI")
    if transport.get("nnodes", 1) not in (0, 1):
        return f"RCCL counted {transport['nnodes']} nodes for {world} ranks of one node"
    return None


# ------------------------------------------------------------------ verification
# Every number the record reports is checked against a stated bound (riemann.cpp:94-96: the
# printed result is the program's contract). For 4/(1+x^2) on [0, 1] the truncation error of
# each rule is known in closed form (Euler-Maclaurin with f(0) - f(1) = 2, f'(1) - f'(0) = -2):
#   left  value - pi = h - h^2/6 + O(h^4)     right  -h - h^2/6     mid  h^2/12
# so a run passes when |err| is that to within 1e-13 (fp64 roundoff of a 1e10-term sum is
# ~1e-15). fp32 runs (fp32 samples, fp64 fold) pass at |err| <= 2h + 1e-10.
PI4_TOL = 1e-13


def pi4_expected_abs_err(rule: str, n: int) -> float:
    h = 1.0 / n
    return {"left": h - h * h / 6, "right": h + h * h / 6, "mid": h * h / 12}[rule]


def verify_rule(integrand: str, rule: str, dtype: str) -> str:
    if integrand == "pi4" and dtype == "fp64":
        return f"| |err| - {rule}-rule truncation | <= {PI4_TOL:g}"
    if dtype == "fp32":
        return "|err| <= 2h + 1e-10"
    if dtype == "fp32acc":
        return "|err| <= 2h + 1e-6 |value| (fp32 accumulation)"
    return "finite; left: |err| <= 4(b-a)/N + 1e-12, else <= 1e-9"


def result_ok(integrand: str, rule: str, dtype: str, n: int, abs_err: float, spec=None) -> bool:
    if not math.isfinite(abs_err):
        return False
    if dtype == "fp32":
        span = (spec.b - spec.a) if spec is not None else 1.0
        return abs_err <= 2.0 * span / n + 1e-10
    if dtype == "fp32acc":
        span = (spec.b - spec.a) if spec is not None else 1.0
        scale = abs(spec.analytic()) if spec is not None else math.pi
        return abs_err <= 2.0 * span / n + 1e-6 * scale
    if integrand == "pi4":
        return abs(abs_err - pi4_expected_abs_err(rule, n)) <= PI4_TOL
    span = (spec.b - spec.a) if spec is not None else 1.0
    return abs_err <= (4.0 * span / n + 1e-12 if rule == "left" else 1e-9)


def _timed_steps(ctx, plan, steps, pipeline, dev, graph_batches: bool = False) -> float:
    """ms per step of `steps` steps in batches (slowest rank), warmed and bracketed: graph
    replays, except a multi-step plan's batches, whose two kernels are launched directly
    (see main) unless graph_batches."""
    import torch

    graphs = graph_batches or not plan.multistep
    if graphs:
        plan.prepare_steps(steps)
    # warm + clock settle: >= 30 ms of the same batches. The count is agreed across ranks
    # (MAX) — every batch holds a collective, so every rank must run the same number.
    t_w = time.perf_counter()
    plan.launch_steps(steps, pipeline, graphs)
    plan.sync()
    per = max(time.perf_counter() - t_w, 1e-6)
    reps = torch.tensor([math.ceil(0.03 / per)], dtype=torch.float64, device=dev)
    ctx.all_reduce_max(reps)
    for _ in range(int(reps.item())):
        plan.launch_steps(steps, pipeline, graphs)
    plan.sync()
    ctx.barrier()
    plan.barrier()  # device barrier (see main's timed region)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan.launch_steps(steps, pipeline, graphs)
    plan.sync()
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / steps * 1e3], dtype=torch.float64, device=dev)
    ctx.all_reduce_max(t)
    return float(t.item())


def single_shot(ctx, kw, args, pipeline, dev, reps: int = 50) -> dict:
    """One pi4 N = 1e9 integration per call, launch to pinned result (median of `reps`).

    One GPU: the plan is built for single integrations (multistep off: the full grid, one
    fused launch whose last workgroup stores the value straight into pinned host memory), and
    RiemannPlan.time_one_shot times four forms in C++: direct (fused launch + stream sync),
    direct_poll (the same launch, the host spinning on the pinned result word), graph /
    graph_poll (a captured 1-step batch replayed). Several GPUs (or --force-collective): one
    step per call through the rank's collective plan (barrier, launch, all-reduce, copy,
    sync), slowest rank."""
    import torch

    from cuda_v_mpi_amd import Integrator

    n1 = 10**9
    want = pi4_expected_abs_err(args.rule, n1)
    rec: dict = {"N": n1, "reps": reps, "n_gpus": ctx.world, "forms": {}}
    if ctx.world == 1 and not args.force_collective:
        one = Integrator("pi4", n=n1, div=args.div, **dict(kw, dtype="fp64", multistep=False))
        p = one.plan
        rec["grid"] = p.grid
        ok = True
        for mode in ("direct_poll", "direct", "graph_poll", "graph"):
            # 400 settling calls of the same form first (from idle the clocks need ~250 to
            # settle: profiles/r4/oneshot_trace.md), then reps timed ones
            r = p.time_one_shot(reps, mode, 400)
            e = abs(r["value"] - math.pi)
            ok = ok and abs(e - want) <= PI4_TOL
            rec["forms"][mode] = {"median_us": r["median_us"], "min_us": r["min_us"],
                                  "max_us": r["max_us"],
                                  "device_median_us": r["device_median_us"],
                                  "result": r["value"]}
        best = min(rec["forms"], key=lambda k: rec["forms"][k]["median_us"])
        rec.update(best_form=best, ms_one_shot=rec["forms"][best]["median_us"] * 1e-3,
                   device_ms_one_shot=rec["forms"][best]["device_median_us"] * 1e-3,
                   verified=bool(ok))
        del one
        return rec
    st = Integrator("pi4", n=n1, div=args.div, **dict(kw, dtype="fp64"))
    p = st.plan
    for _ in range(20):  # warm: code objects, RCCL connections, clocks
        p.run_steps(1, pipeline, False)
    walls, devs = [], []
    for _ in range(reps):
        t = p.run_steps(1, pipeline, False)  # barrier inside: every rank starts together
        walls.append(t["wall_s"] * 1e6)
        devs.append(t["device_ms"] * 1e3)
    walls.sort()
    devs.sort()
    m = torch.tensor([walls[reps // 2], devs[reps // 2]], dtype=torch.float64, device=dev)
    ctx.all_reduce_max(m)
    v = p.host_result(p.host_index_of(0, False))
    e = abs(v - math.pi)
    rec["forms"]["collective_step"] = {"median_us": float(m[0]), "device_median_us": float(m[1]),
                                       "result": v}
    rec.update(best_form="collective_step", ms_one_shot=float(m[0]) * 1e-3,
               device_ms_one_shot=float(m[1]) * 1e-3, grid=p.grid,
               verified=bool(abs(e - want) <= PI4_TOL))
    del st
    return rec


def run_extras(args, ctx, integ, n_total, pipeline, dev) -> dict:
    """Measured after (never inside) the timed region; every rank takes part. Every plan here
    shares the headline's native communicator (one RCCL communicator per rank)."""
    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.ops import kernels

    out: dict = {}
    comm = getattr(integ, "_comm", None)
    kw = dict(rule=args.rule, dtype=args.dtype, ctx=ctx, comm=args.comm, slots=args.slots,
              bucket=not args.no_bucket, force_collective=args.force_collective,
              comm_obj=comm, step_streams=args.step_streams,
              multistep=not args.no_multistep)
    pi4 = args.integrand == "pi4"
    # (1) the same config with correctly rounded division for every sample
    if pi4 and args.div != "ieee":
        ie = Integrator(args.integrand, n=n_total, div="ieee", **kw)
        steps = 40
        ms = _timed_steps(ctx, ie.plan, steps, pipeline, dev, args.graph_batches)
        v = ie.plan.host_result(ie.plan.host_index_of(steps - 1, True))
        e = abs(v - math.pi)
        out["ieee_div"] = {"value": n_total / (ms * 1e-3), "ms_per_step": ms, "steps": steps,
                           "result": v, "abs_err": e,
                           "verified": result_ok("pi4", args.rule, args.dtype, n_total, e)}
        out["ieee_div_value"] = out["ieee_div"]["value"]
        del ie
    # (2) per-point accuracy of the division the headline used, on two 64 K-sample windows of
    #     this rank's slice (its first samples, and 1/8 in; rank 0's are reported): against
    #     the IEEE path's own values, and against the true value 4/(1 + x^2) at the true
    #     coordinate in x87 extended precision (profiles/r5/accuracy_ab.md)
    eff = str(integ.plan.effective_div).split(".")[-1]
    b0, cnt = integ.plan.begin, integ.plan.count
    w = min(1 << 16, cnt)
    windows = [b0, b0 + cnt // 8 + 12_345] if cnt >= 8 * w else [b0]

    def ulps(div):  # every point of the windows: |value - reference| in ulps
        import numpy as np
        import torch

        u_all, t_all, per = [], [], []
        # the kernels' own step (fp64 (b - a) / N) and the true coordinate a + (i + off) h
        h = np.longdouble(float((integ.spec.b - integ.spec.a) / n_total))
        off = {"left": 0.0, "mid": 0.5, "right": 1.0}[args.rule]
        for i0 in windows:
            v = kernels.point_values(integ.spec, n_total, rule=args.rule, div=div, i_begin=i0,
                                     n_local=w)
            r = kernels.point_values(integ.spec, n_total, rule=args.rule, div="ieee",
                                     i_begin=i0, n_local=w)
            spacing = torch.nextafter(r.abs(), torch.full_like(r, math.inf)) - r.abs()
            u = ((v - r) / spacing).abs().cpu().numpy()
            x = np.longdouble(integ.spec.a) + (np.arange(w, dtype=np.longdouble) +
                                               np.longdouble(i0) + np.longdouble(off)) * h
            true = np.longdouble(4) / (np.longdouble(1) + x * x)
            t = np.abs((v.cpu().numpy().astype(np.longdouble) - true) /
                       np.spacing(true.astype(np.float64)).astype(np.longdouble)).astype(np.float64)
            u_all.append(u)
            t_all.append(t)
            per.append({"i0": int(i0), "max_ulp": float(u.max()), "vs_true_max_ulp": float(t.max()),
                        "vs_true_mean_ulp": float(t.mean())})
        u, t = np.concatenate(u_all), np.concatenate(t_all)
        return {"max_ulp": float(u.max()), "frac_within_1ulp": float((u <= 1.0).mean()),
                "frac_within_2ulp": float((u <= 2.0).mean()),
                "vs_true_max_ulp": float(t.max()), "vs_true_mean_ulp": float(t.mean()),
                "vs_true_frac_within_1ulp": float((t <= 1.0).mean()),
                "window": [int(windows[-1]), int(w)], "windows": per}

    # per-point bounds. series_exact is checked against the TRUE value
    # (<= 1.5 ulp, as test_pi4_series_exact_per_point_accuracy; measured max 1.42): against
    # the IEEE path's own values both sides round independently (series_exact up to ~1.42
    # ulp from the true value, IEEE division up to ~1.57), so the two may sit 3 ulp apart
    # where neither is wrong — that comparison is reported, bounded by 3. The g-fold of
    # series rounds every sample at ulp(1/2): within 5 of IEEE.
    bound = {"series_exact": 3.0}.get(eff, 5.0)
    true_bound = {"series_exact": 1.5}.get(eff)
    if pi4 and args.dtype == "fp64" and eff != "ieee":
        pp = ulps(eff)
        good = pp["max_ulp"] <= bound and (true_bound is None or
                                           pp["vs_true_max_ulp"] <= true_bound)
        out["per_point"] = dict(pp, division=eff, bound_max_ulp=bound,
                                bound_vs_true_max_ulp=true_bound, verified=bool(good))
        out["per_point_max_ulp"] = out["per_point"]["max_ulp"]
        out["per_point_frac_within_1ulp"] = out["per_point"]["frac_within_1ulp"]
        out["per_point_vs_true_max_ulp"] = out["per_point"]["vs_true_max_ulp"]
        out["per_point_window"] = out["per_point"]["window"]
    # (2b) the same config with the other series form: under the default series_exact
    #      headline (per point as accurate as IEEE division), the g = 1/2 + e fold ("series":
    #      one square per sample rounded at ulp(1/2), up to 5 ulp per point) — what the
    #      headline's exact-grade points cost in speed; under --div series, series_exact.
    if pi4 and args.dtype == "fp64" and args.div in ("series", "series_exact"):
        alt = "series" if args.div == "series_exact" else "series_exact"
        ex = Integrator(args.integrand, n=n_total, div=alt, **kw)
        steps = 48
        ms = _timed_steps(ctx, ex.plan, steps, pipeline, dev, args.graph_batches)
        v = ex.plan.host_result(ex.plan.host_index_of(steps - 1, True))
        e = abs(v - math.pi)
        ab = {"series_exact": 3.0}.get(alt, 5.0)
        pp = ulps(alt)
        out[f"{alt}_div"] = {
            "value": n_total / (ms * 1e-3), "ms_per_step": ms, "steps": steps, "result": v,
            "abs_err": e, "division": str(ex.plan.effective_div).split(".")[-1],
            "per_point": dict(pp, bound_max_ulp=ab),
            "verified": bool(result_ok("pi4", args.rule, args.dtype, n_total, e) and
                             pp["max_ulp"] <= ab and
                             (alt != "series_exact" or pp["vs_true_max_ulp"] <= 1.5))}
        del ex
    # (3) the headline config in its other scaling form. Strong headline (the default: N = 1e9
    #     IN TOTAL, riemann.cpp:10,71-73): the weak form, 1e9 samples PER GPU (N = 1e9 x G,
    #     "weak_1e9_per_gpu"). Weak headline (--scaling weak): the metric's fixed N = 1e9 split
    #     over the ranks ("strong_1e9"). Own graph and timing; equal configs at G = 1.
    if pi4:
        weak_extra = args.scaling == "strong"
        key, n1 = ("weak_1e9_per_gpu", 10**9 * ctx.world) if weak_extra else ("strong_1e9", 10**9)
        st = Integrator("pi4", n=n1, div=args.div, **dict(kw, dtype="fp64"))
        steps = 48
        ms = _timed_steps(ctx, st.plan, steps, pipeline, dev, args.graph_batches)
        v = st.plan.host_result(st.plan.host_index_of(steps - 1, True))
        e = abs(v - math.pi)
        out[key] = {"N": n1, "value": n1 / (ms * 1e-3), "ms_per_step": ms,
                    "steps": steps, "result": v, "abs_err": e,
                    "n_per_gpu": st.plan.count, "grid": st.plan.grid,
                    "scaling": "weak" if weak_extra else "strong", "n_gpus": ctx.world,
                    "verified": result_ok("pi4", args.rule, "fp64", n1, e)}
        del st
    # (4) BASELINE config #3: N = 1e10 in total over the same GPUs (strong scaling)
    if pi4:
        n3 = 10**10
        st = Integrator("pi4", n=n3, div=args.div, **dict(kw, dtype="fp64"))
        steps = 20
        ms = _timed_steps(ctx, st.plan, steps, pipeline, dev, args.graph_batches)
        v = st.plan.host_result(st.plan.host_index_of(steps - 1, True))
        e = abs(v - math.pi)
        out["baseline3_strong_1e10"] = {"N": n3, "value": n3 / (ms * 1e-3), "ms_per_step": ms,
                                        "steps": steps, "result": v, "abs_err": e,
                                        "n_per_gpu": st.plan.count, "scaling": "strong",
                                        "verified": result_ok("pi4", args.rule, "fp64", n3, e)}
        del st
    # (5) BASELINE config #5: the 2-D field v(x) v(y) from the velocity profile, 4096^2
    #     bilinear midpoint samples, sample rows split over the same GPUs; one integration =
    #     one multi-step launch per graph replay of p2.graph_steps integrations (the replay
    #     size rule is table2d_auto_graph_steps: about Table2DPlan::kReplaySamples = 2^33
    #     samples per replay, 512 integrations for the whole field, up to 1024 for a small
    #     row share), the replay's per-integration partials meeting in one RCCL all-reduce
    #     (Table2DPlan) on the shared communicator
    if pi4:
        import torch

        from cuda_v_mpi_amd import native

        m = native()
        g = 4096
        p2 = m.Table2DPlan(g, 1800.0, ctx.device, comm, not args.no_bucket,
                           multistep=not args.no_multistep)
        p2.run()
        # each time() call first replays ~30 ms untimed (steady clocks); best of 3
        ms = min(p2.time(p2.graph_steps * 10, True) for _ in range(3))
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        ctx.all_reduce_max(t)
        ms = float(t.item())
        v, want = p2.last_result(), m.table2d_oracle(g)
        rel = abs(v - want) / want
        out["baseline5_table2d_4096"] = {
            "grid": g, "samples": g * g, "ms_per_integration": ms,
            "samples_per_s": g * g / (ms * 1e-3), "result": v, "midpoint_oracle": want,
            "rel_err_vs_oracle": rel, "rows_this_rank": [p2.row0, p2.row1],
            "bucketed_allreduce": bool(p2.bucketed), "n_gpus": ctx.world,
            "step_streams": p2.step_streams, "multistep": bool(p2.multistep),
            "phases": p2.phases, "workgroups": p2.workgroups, "graph_steps": p2.graph_steps,
            "verified": bool(rel <= 1e-12)}
        del p2
    # (6) BASELINE config #4: the same integral through the packed-fp32 path. Samples are
    #     evaluated in packed fp32; each 192-sample tile's value is folded into an fp64 lane
    #     accumulator and the DPP/LDS reduction runs in fp64 ("accum": "fp64-fold": an fp32
    #     fold biases the sum by -8e-9 relative at N = 1e9, riemann.cpp's Pi4F32 notes;
    #     the all-fp32 variant is measured in profiles/r3/fp32_accum.jsonl)
    if pi4 and args.dtype == "fp64":
        f32 = Integrator("pi4", n=n_total, div=args.div, **dict(kw, dtype="fp32"))
        # two full 48-step batches: a batch's fixed cost (~28 us: launch, ramp, tail, close,
        # syncs; profiles/r4/replay_overhead.jsonl) is 1.8 % of a 40-step fp32 batch
        steps = 96
        ms = _timed_steps(ctx, f32.plan, steps, pipeline, dev, args.graph_batches)
        v = f32.plan.host_result(f32.plan.host_index_of(steps - 1, True))
        ref = integ.plan.host_result(integ.plan.host_index_of(0, True))
        e, rd = abs(v - math.pi), abs(v - ref) / abs(ref)
        out["baseline4_fp32"] = {"value": n_total / (ms * 1e-3), "ms_per_step": ms,
                                 "steps": steps, "result": v, "abs_err": e,
                                 "rel_diff_vs_fp64": rd, "dtype": "fp32", "accum": "fp64-fold",
                                 "verified": bool(rd <= 1e-9 and
                                                  result_ok("pi4", args.rule, "fp32", n_total, e))}
        del f32
        # ... and with fp32 accumulation down to the workgroup partial (fp32 lane sums,
        # v_add_f32_dpp wave reduction, fp32 LDS step): the all-fp32 reduction the config
        # names, kept as the measured alternative (bound: fp32-level agreement, 1e-6)
        fa = Integrator("pi4", n=n_total, div=args.div, **dict(kw, dtype="fp32acc"))
        ms = _timed_steps(ctx, fa.plan, steps, pipeline, dev, args.graph_batches)
        v = fa.plan.host_result(fa.plan.host_index_of(steps - 1, True))
        e, rd = abs(v - math.pi), abs(v - ref) / abs(ref)
        out["baseline4_fp32_accum32"] = {"value": n_total / (ms * 1e-3), "ms_per_step": ms,
                                         "steps": steps, "result": v, "abs_err": e,
                                         "rel_diff_vs_fp64": rd, "dtype": "fp32",
                                         "accum": "fp32", "verified": bool(rd <= 1e-6)}
        del fa
    # (6b) one integration per call — the reference's own timing unit (cintegrate.cu:102-104,
    #      127-141 and riemann.cpp:49-51,90-93 clock exactly one run): pi4 N = 1e9 IN TOTAL,
    #      from the launch call to the result in pinned host memory, median of 50 calls
    if pi4 and args.dtype == "fp64":
        out["single_shot_1e9"] = single_shot(ctx, kw, args, pipeline, dev)
    # (6c) the reference's own integrands (sin: riemann.cpp:37, cintegrate.cu:68; the table
    #      interpolant: cintegrate.cu:36-44; the analytic train model: riemann.cpp:103-116) and
    #      the random-coefficient polynomial, each one timed 48-step graph batch of the same
    #      shape as the headline (the headline's N), checked against its analytic value
    if pi4:
        for name in ("sin", "train", "table", "poly"):
            it = Integrator(name, n=n_total, **dict(kw, dtype="fp64"))
            steps = 48
            ms = _timed_steps(ctx, it.plan, steps, pipeline, dev, args.graph_batches)
            v = it.plan.host_result(it.plan.host_index_of(steps - 1, True))
            e = abs(v - it.spec.analytic())
            out[f"integrand_{name}"] = {
                "N": n_total, "value": n_total / (ms * 1e-3), "ms_per_step": ms, "steps": steps,
                "result": v, "abs_err": e, "domain": [it.spec.a, it.spec.b],
                "multistep": bool(it.plan.multistep), "grid": it.plan.grid,
                "verified": result_ok(name, args.rule, "fp64", n_total, e, it.spec)}
            del it
    # (7) BASELINE config #1: the serial CPU sum at N = 1e6 (the reference's plumbing case),
    #     on one host thread of the native host engine
    if pi4:
        from cuda_v_mpi_amd import native as _native

        mm = _native()
        c1 = Integrator("pi4", n=10**6, rule=args.rule, backend="host", threads=1)
        best1 = min(c1.run().seconds_device for _ in range(3))
        v1 = c1.run().value
        e1 = abs(v1 - math.pi)
        out["baseline1_serial_cpu_1e6"] = {"N": 10**6, "value": 10**6 / best1,
                                           "ms": best1 * 1e3, "result": v1, "abs_err": e1,
                                           "threads": 1, "isa": mm.host_isa(),
                                           "verified": result_ok("pi4", args.rule, "fp64",
                                                                 10**6, e1)}
    # (8) the reference's own side of its CUDA-vs-MPI comparison: the same integral on this
    #     node's host cores (native host engine, per-sample fp64 vector threads, each rank
    #     its slice with its share of the cores, best of 3, slowest rank)
    import torch

    from cuda_v_mpi_amd import native

    m = native()
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", ctx.world)))
    # torch.distributed.run sets OMP_NUM_THREADS=1 for every rank when it starts several per
    # node and the variable was unset: that is its default, not a share someone chose, so
    # the ranks then split this process's CPU affinity instead
    torchrun_default = ("TORCHELASTIC_RUN_ID" in os.environ and local > 1 and
                        os.environ.get("OMP_NUM_THREADS") == "1" and
                        not os.environ.get("MIINT_HOST_THREADS"))
    share_given = not torchrun_default and \
        any(os.environ.get(k) for k in ("MIINT_HOST_THREADS", "OMP_NUM_THREADS"))
    if torchrun_default:
        threads = max(1, len(os.sched_getaffinity(0)) // local)
    else:
        threads = m.HostPool.default_threads() if share_given else \
            max(1, m.HostPool.default_threads() // local)
    host = Integrator(args.integrand, n=n_total, rule=args.rule, backend="host", ctx=ctx,
                      threads=threads)
    host.run()  # warm: threads, pages
    best = min(host.run().seconds_device for _ in range(3))
    t = torch.tensor([best], dtype=torch.float64, device=dev)
    ctx.all_reduce_max(t)
    v = host.run().value
    e = abs(v - host.spec.analytic())
    out["host_engine"] = {"value": n_total / float(t.item()), "ms": float(t.item()) * 1e3,
                          "ranks": ctx.world, "threads_per_rank": threads,
                          "isa": m.host_isa(), "result": v, "abs_err": e,
                          "verified": result_ok(args.integrand, args.rule, "fp64", n_total, e,
                                                host.spec)}
    return out


if __name__ == "__main__":
    sys.exit(main())
