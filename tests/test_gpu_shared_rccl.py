"""Multi-rank RCCL on one GPU: W processes share device 0 (MIINT_OVERSUBSCRIBE=1,
miint/comm.hpp ranks_share_devices). Each rank names itself a host of its own, so RCCL builds
real world-W communicators (nNodes = W) and carries the collectives over its socket transport
on loopback. This runs the code the 8-GPU node runs — unique-id rendezvous, ncclCommInitRank,
all-reduce / all-gather captured in hipGraphs — with RCCL instead of the LoopbackComm; only the
transport differs (sockets instead of xGMI), and the records say so (rccl_transport, nnodes).

What is asserted about the multi-rank numbers: every native tool starts its
ranks' clocks behind a collective barrier and reports the slowest rank's time (RankAgree), so
W ranks sharing ONE GPU can never report more than one GPU's rate; a rank made slow on
purpose (MIINT_FAULT_RANK / MIINT_FAULT_DELAY_MS) sets rank 0's reported time; a scan timeout
forced on rank 1 is every rank's exit status 3; and riemann --parity is the reference's
master/worker program run by P real RCCL ranks (riemann.cpp:62-86).
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
sys.path.insert(0, REPO)

from bench import rendezvous_port  # noqa: E402


def _env(**extra):
    e = dict(os.environ, MIINT_OVERSUBSCRIBE="1", **extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    return e


def _proc(args, timeout=150, **env):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=_env(**env),
                          cwd=REPO)


def _records(args, timeout=150, **env):
    p = _proc(args, timeout, **env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def _np(w, *prog):
    return [os.path.join(BIN, "miintrun"), "-np", str(w), "--", *prog]


def _shared_rccl(rec, world):
    """The record names how its ranks met: W RCCL ranks on one GPU, over sockets."""
    assert rec["comm"] == "rccl" and rec["rccl_world"] == world
    assert rec["ranks_share_gpus"] is True
    assert rec["rccl_transport"].startswith("NET/Socket") and rec["rccl_nnodes"] == world
    # sockets are this setup's transport, so the fail-closed check exempts it (and says so)
    assert rec["transport_verified"] is True and "transport_error" not in rec


@pytest.mark.parametrize("world", [2, 4])
def test_riemann_ranks_share_gpu_over_rccl(cuda, world):
    one = _records([os.path.join(BIN, "riemann"), "--integrand", "pi4", "--n", "1e9",
                    "--iters", "20", "--json"])[0]
    rec = _records(_np(world, os.path.join(BIN, "riemann"), "--integrand", "pi4", "--n", "1e9",
                       "--iters", "20", "--json"))
    assert len(rec) == 1 and rec[0]["gpus"] == world  # rank 0 prints
    _shared_rccl(rec[0], world)
    # N = 1e9 split over the ranks, summed by RCCL: the left-rule truncation h
    assert abs(rec[0]["abs_err"] - 1e-9) < 1e-13
    # W ranks on ONE GPU: barrier before every rank's clock + the slowest rank's time, so the
    # job can never beat the GPU's single-rank rate (round 3 reported 1.7-2.6x it)
    assert rec[0]["subintervals_per_s"] <= 1.05 * one["subintervals_per_s"], (rec[0], one)


def test_slow_rank_sets_rank0_time_over_rccl(cuda):
    """Rank 1 holds its end-of-timing event back by 300 ms (after the last collective of the
    timed region): rank 0's own interval is unchanged, so only the max over ranks shows it."""
    args = _np(2, os.path.join(BIN, "riemann"), "--integrand", "pi4", "--n", "1e8", "--iters", "1",
               "--json", "--no-one-shot")
    slow = _records(args, MIINT_FAULT_RANK="1", MIINT_FAULT_DELAY_MS="300")[0]
    fast = _records(args)[0]
    assert slow["device_ms"] >= 300.0 and fast["device_ms"] < 300.0
    assert slow["result"] == fast["result"]


def test_trainscan_ranks_share_gpu_over_rccl(cuda):
    one = _records([os.path.join(BIN, "trainscan"), "--iters", "3", "--json"])[0]
    two = _records(_np(2, os.path.join(BIN, "trainscan"), "--iters", "3", "--json"))[0]
    assert two["gpus"] == 2 and two["timeout"] == 0 and two["timeout_ranks"] == 0
    _shared_rccl(two, 2)
    assert abs(two["distance"] - one["distance"]) <= 1e-9 * abs(one["distance"])


def test_trainscan_timeout_on_rank1_is_every_ranks_exit_3(cuda):
    """A hand-off spin timeout reported by rank 1 only (forced): the flag is all-reduced
    before any rank enters another collective, every rank exits 3, rank 0 says so."""
    p = _proc(_np(2, os.path.join(BIN, "trainscan"), "--json"), MIINT_FAULT_RANK="1",
              MIINT_FAULT_SCAN_TIMEOUT="1")
    assert p.returncode == 3, (p.stdout[-2000:], p.stderr[-2000:])
    rec = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(rec) == 1 and rec[0]["timeout"] == 1 and rec[0]["timeout_ranks"] == 1
    assert "hit its limit on 1 of 2 rank(s)" in p.stderr


def test_cintegrate_and_miint_ranks_share_gpu(cuda):
    c = _records(_np(2, os.path.join(BIN, "cintegrate"), "--json"))[0]
    _shared_rccl(c, 2)
    assert abs(c["result"] - 122000.004) < 1e-6
    # both runs settled (~60 ms of steps, the default): a 20-step settle left the one-rank
    # run inside the clock ramp (1.04e13) while the two ranks' longer run was past it
    # (1.12e13 aggregate), which flipped this sanity check once
    b = _records(_np(2, os.path.join(BIN, "miint"), "bench", "--integrand", "pi4", "--iters",
                     "200"))[0]
    _shared_rccl(b, 2)
    one = _records([os.path.join(BIN, "miint"), "bench", "--integrand", "pi4", "--iters",
                    "200"])[0]
    assert b["subintervals_per_s"] <= 1.05 * one["subintervals_per_s"], (b, one)


def test_table2d_two_ranks_reports_the_chains_it_ran(cuda):
    """the bucketed two-rank plan must run (and report) the chain count its
    construction chose, not one decided before it knew it was bucketed."""
    r = _records(_np(2, os.path.join(BIN, "miint"), "table2d", "--grid", "4096", "--iters", "64",
                     "--no-multistep"))[0]
    _shared_rccl(r, 2)
    assert r["chained"] and r["bucketed_allreduce"]
    assert r["step_streams"] == 2  # kAutoT2Streams, now in effect on a bucketed plan
    assert r["rel_err_vs_oracle"] < 1e-12


def test_bench_two_ranks_native_rccl_one_gpu(cuda):
    """Two ranks on the one GPU over RCCL's socket transport: the record, the all-reduce into
    pinned host memory, and the untimed diagnostic batch (compute, tail, per-rank max / min,
    the communicator's 8-byte all-reduce latency and allgather bandwidth, RCCL's channel
    lines)."""
    rec = _records([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "10",
                    "--warmup", "3", "--no-extras", "--diag-allgather-mb", "16"], timeout=240)
    assert len(rec) == 1
    r = rec[0]
    assert r["verified"] and r["n_gpus"] == 2 and r["ranks_share_gpus"]
    assert r["rccl_world"] == 2 and r["native_rccl_comms"] == 1 and r["torch_nccl_groups"] == 0
    assert r["rccl_transport"] == "NET/Socket" and r["rccl_nnodes"] == 2
    assert r["transport_verified"] and r["transport_error"] is None
    assert r["comm_fallback"] is None and r["config"]["batch_launch"] == "direct"
    assert r["direct_steps_timed"] == 10 and r["config"]["multistep"]
    # the host barrier moved before the re-arm batch; the RCCL barrier stands before the clock
    assert r["warmup_rearm_batch"] and r["pre_clock_barrier"] == "device"
    assert r["config"]["bucketed_allreduce"] and r["config"]["N"] == 10**9
    assert r["config"]["n_per_gpu"] == 5 * 10**8 and r["scaling"] == "strong"
    assert r["native_comm_verified"] and r["config"]["allreduce_to_host"]
    d = r["diagnostic_batch"]
    assert d["path"] == "native" and d["steps"] == 10 and d["allreduce_to_host"]
    for k in ("compute_us", "tail_us", "boundary_us", "allreduce_us", "device_us", "wall_us",
              "host_us"):
        assert len(d[k]["per_rank"]) == 2 and d[k]["max"] >= d[k]["min"], k
    assert d["compute_us"]["min"] > 0 and d["allreduce_us"]["max"] > 0
    assert d["comm"]["transport"] == "rccl" and d["comm"]["allreduce_8b_us"] > 0
    assert d["comm"]["allgather_busbw_gbs"] > 0 and d["comm"]["allgather_bytes"] == 16_000_000
    assert d["rccl_init"]["channels"] and d["rccl_init"]["lines"]


def test_bench_driver_launch_form_two_ranks(cuda):
    """The driver's own launch line (torch.distributed.run, one rank per process) with the
    two ranks on the one GPU: the record is rank 0's, with the max over ranks."""
    rec = _records([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                    str(rendezvous_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                    "--steps", "10", "--warmup", "3", "--no-extras"], timeout=240)
    assert len(rec) == 1
    r = rec[0]
    assert r["launcher"] == "torchrun" and r["verified"] and r["rccl_world"] == 2
    assert abs(r["ms_per_step"] - max(r["per_rank_ms"])) <= 1e-9


@pytest.mark.parametrize("algo", ["fused", "lookback"])
def test_trainscan_parity_seven_rccl_ranks(cuda, algo):
    """4main.c at P = 7 prints 0.000000 (its fill/scan partitions disagree): the
    GPU plan reproduces it with seven real RCCL ranks (allgather-fed carries)."""
    p = _proc(_np(7, os.path.join(BIN, "trainscan"), "--parity", "--algo", algo), timeout=200)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l.strip() for l in p.stdout.splitlines()]
    assert "Step size of 10000" in lines, p.stdout[-3000:]
    assert "Total distance traveled = 0.000000" in lines, p.stdout[-3000:]


@pytest.mark.parametrize("world", [3, 7])
def test_riemann_parity_is_a_distributed_master_worker_run(cuda, world):
    """riemann --parity under P RCCL ranks is the reference's program (riemann.cpp:62-86):
    rank 0 coordinates (partial 0), rank r >= 1 integrates worker r-1's (int)(N/W) samples,
    one allgather of the partials, rank 0 adds them in rank order. The value agrees with the
    host emulation of the reference (its sequential fp64 sums: roundoff ~1e-12)."""
    n = 10**8
    rec = _records(_np(world, os.path.join(BIN, "riemann"), "--parity", "--n", str(n), "--json"),
                   timeout=200)
    assert len(rec) == 1
    r = rec[0]
    assert r["parity"] and r["gpus"] == world
    _shared_rccl(r, world)
    W = world - 1
    assert r["workers"] == W and r["samples"] == W * (n // W)
    parts = r["partials"]
    assert len(parts) == world and parts[0] == 0.0
    acc = 0.0
    for q in range(1, world):  # the MPI_Recv loop's order and rounding, bit for bit
        acc += parts[q]
    assert acc == r["result"]
    # each worker's partial is that slice's integral; together the left-rule sum of sin
    host = _records([os.path.join(BIN, "riemann"), "--device", "cpu", "--parity", "--ranks",
                     str(world), "--n", str(n), "--json"], timeout=200)[0]
    assert abs(r["result"] - host["result"]) < 1e-10
    assert abs(r["result"] - 2.0) < 1e-8
    # the slices: worker w integrates [w pi/W, (w+1) pi/W)
    for w in range(W):
        exact = math.cos(w * math.pi / W) - math.cos((w + 1) * math.pi / W)
        assert abs(parts[w + 1] - exact) < 1e-7


def test_trainscan_replicate_ranks_share_gpu(cuda):
    """trainscan --replicate under 2 RCCL ranks (4main.c:157): the 144 MB allgather leaves
    both ranks with bitwise-equal copies that match the one-rank table within roundoff."""
    one = _records([os.path.join(BIN, "trainscan"), "--replicate", "--json"])[0]
    assert one["replicate"] and one["replicas_identical"] and one["replica_n"] == 18_000_000
    two = _records(_np(2, os.path.join(BIN, "trainscan"), "--replicate", "--json"))[0]
    _shared_rccl(two, 2)
    assert two["replicas_identical"] is True and two["replica_n"] == 18_000_000
    assert two["replica_sum"] == pytest.approx(one["replica_sum"], rel=1e-12)
    for x, y in zip(two["replica_at"], one["replica_at"]):
        assert x == pytest.approx(y, rel=1e-12, abs=1e-9)


def test_miint_comm_ranks_share_gpu(cuda):
    """miint comm as 2 RCCL processes on the one GPU: every collective size reports a time,
    the transport is the sockets this setup uses, and the record names it."""
    p = _proc(_np(2, os.path.join(BIN, "miint"), "comm", "--max-bytes", "1e6", "--iters", "3"))
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert {r["op"] for r in rows} == {"allreduce", "allgather", "broadcast"}
    for r in rows:
        assert r["gpus"] == 2 and r["us"] > 0 and r["ranks_share_gpus"] is True
        assert r["rccl_transport"].startswith("NET/Socket") and r["transport_verified"]
