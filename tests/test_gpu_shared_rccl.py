"""Multi-rank RCCL on one GPU: W processes share device 0 (MIINT_OVERSUBSCRIBE=1,
miint/comm.hpp ranks_share_devices). Each rank names itself a host of its own, so RCCL builds
real world-W communicators (nNodes = W) and carries the collectives over its socket transport
on loopback. This runs the code the 8-GPU node runs — unique-id rendezvous, ncclCommInitRank,
all-reduce / all-gather captured in hipGraphs, the max-over-ranks timing — with RCCL instead of
the LoopbackComm; only the transport differs (sockets instead of xGMI).

The reference's multi-process side is MPI (riemann.cpp:62-86, 4main.c:69-71 + 157-236); the
values checked here are the single-rank ones, which the oracles pin elsewhere.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")


def _env():
    # RCCL's warnings go to a file: on the ranks' shared stdout they split the output lines
    e = dict(os.environ, MIINT_OVERSUBSCRIBE="1", NCCL_DEBUG="WARN", NCCL_DEBUG_FILE=os.devnull)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    return e


def _records(args, timeout=150):
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=_env(), cwd=REPO)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def _np(w, *prog):
    return [os.path.join(BIN, "miintrun"), "-np", str(w), "--", *prog]


@pytest.mark.parametrize("world", [2, 4])
def test_riemann_ranks_share_gpu_over_rccl(cuda, world):
    rec = _records(_np(world, os.path.join(BIN, "riemann"), "--integrand", "pi4", "--n", "1e8",
                       "--iters", "5", "--json"))
    assert len(rec) == 1 and rec[0]["gpus"] == world  # rank 0 prints
    # N = 1e8 split over the ranks, summed by RCCL: the left-rule truncation h
    assert abs(rec[0]["abs_err"] - 1e-8) < 1e-13


def test_trainscan_ranks_share_gpu_over_rccl(cuda):
    one = _records([os.path.join(BIN, "trainscan"), "--iters", "1", "--json"])[0]
    two = _records(_np(2, os.path.join(BIN, "trainscan"), "--iters", "1", "--json"))[0]
    assert two["gpus"] == 2 and two["timeout"] == 0
    assert abs(two["distance"] - one["distance"]) <= 1e-9 * abs(one["distance"])


def test_bench_two_ranks_native_rccl_one_gpu(cuda):
    rec = _records([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "10",
                    "--warmup", "3", "--no-extras"], timeout=240)
    assert len(rec) == 1
    r = rec[0]
    assert r["verified"] and r["n_gpus"] == 2 and r["ranks_share_gpus"]
    assert r["rccl_world"] == 2 and r["native_rccl_comms"] == 1 and r["torch_nccl_groups"] == 0
    assert r["comm_fallback"] is None and r["graph_replays_timed"] == 1
    assert r["config"]["bucketed_allreduce"] and r["config"]["N"] == 2 * 10**9


def test_bench_driver_launch_form_two_ranks(cuda):
    """The driver's own launch line (torch.distributed.run, one rank per process) with the
    two ranks on the one GPU: the record is rank 0's, with the max over ranks."""
    rec = _records([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                    "29641", os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "10",
                    "--warmup", "3", "--no-extras"], timeout=240)
    assert len(rec) == 1
    r = rec[0]
    assert r["launcher"] == "torchrun" and r["verified"] and r["rccl_world"] == 2
    assert abs(r["ms_per_step"] - max(r["per_rank_ms"])) <= 1e-9


@pytest.mark.parametrize("algo", ["fused", "lookback"])
def test_trainscan_parity_seven_rccl_ranks(cuda, algo):
    """4main.c at P = 7 prints 0.000000 (its fill/scan partitions disagree): the
    GPU plan reproduces it with seven real RCCL ranks (allgather-fed carries)."""
    p = subprocess.run(_np(7, os.path.join(BIN, "trainscan"), "--parity", "--algo", algo),
                       capture_output=True, text=True, timeout=200, env=_env(), cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l.strip() for l in p.stdout.splitlines()]
    assert "Step size of 10000" in lines, p.stdout[-3000:]
    assert "Total distance traveled = 0.000000" in lines, p.stdout[-3000:]


def test_riemann_parity_master_worker_rccl_equals_loopback(cuda):
    """riemann --parity: P - 1 workers of (int)(N / W) samples each, rank 0 idle
    (riemann.cpp:65-86) — the same value over RCCL ranks as over the loopback transport."""
    args = ["--parity", "--n", "1e8", "--json"]
    lb = _records([os.path.join(BIN, "riemann"), *args, "--loopback", "3"])[0]
    rc = _records(_np(3, os.path.join(BIN, "riemann"), *args))[0]
    assert rc["gpus"] == 3 and rc["parity"]
    assert rc["result"] == pytest.approx(lb["result"], rel=1e-15, abs=0)
