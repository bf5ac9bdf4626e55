"""Multi-GPU tests (SURVEY §7.4 "Comm tests ... 2/4/8 when available"): run only where the
box shows at least that many HIP devices, and compare with the single-GPU result.

The gpurun pool gives one GPU: there these skip, and the 1-rank RCCL graph path
(tests/test_gpu_runtime.py::test_plan_rccl_stage_on_one_gpu), the shared-GPU RCCL variants
(tests/test_gpu_shared_rccl.py) plus the gloo tests carry the multi-rank logic.

Every multi-rank record on distinct GPUs must also SHOW that its ranks met over xGMI
peer-to-peer: RCCL's INIT log names a P2P transport, counts one node, and the
record's own fail-closed verdict (transport_verified) agrees.
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


def _devices() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


def _port() -> int:
    from bench import rendezvous_port  # below the ephemeral range (no self-connect)

    return rendezvous_port()


def _run(args, timeout=600):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ))


def _rec(p):
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    return json.loads([l for l in p.stdout.strip().splitlines() if l.startswith("{")][-1])


def _xgmi(rec, g):
    """The record's ranks are G RCCL ranks on distinct GPUs of one node, met over P2P."""
    assert rec["rccl_world"] == g, rec
    assert rec["rccl_transport"].startswith("P2P"), rec["rccl_transport"]
    assert "NET/" not in rec["rccl_transport"] and rec["rccl_nnodes"] == 1
    assert rec["ranks_share_gpus"] is False and rec["transport_verified"] is True


def _np(g, *prog):
    return [os.path.join(BIN, "miintrun"), "-np", str(g), "--", *prog]


@pytest.mark.parametrize("g", [2, 4, 8])
def test_cli_threads_ncclcomminitall(native, cuda, slice_tol, g):
    """One process driving G GPUs (ncclCommInitAll + threads): the global sum of the G
    rank slices equals the 1-GPU integration of the same N to fp64 roundoff."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    one = _run([os.path.join(BIN, "riemann"), "--integrand", "pi4", "--rule", "mid", "--json"])
    many = _run([os.path.join(BIN, "riemann"), "--integrand", "pi4", "--rule", "mid", "--json",
                 "--gpus", str(g)])
    assert one.returncode == 0 and many.returncode == 0, many.stderr[-2000:]
    a = json.loads(one.stdout.strip().splitlines()[-1])["result"]
    rb = json.loads(many.stdout.strip().splitlines()[-1])
    _xgmi(rb, g)
    assert rb["result"] == pytest.approx(a, rel=slice_tol(g), abs=0)


@pytest.mark.parametrize("g,graphs", [(2, False), (8, False), (8, True)])
def test_bench_torchrun_rccl(native, cuda, g, graphs):
    """bench.py under torchrun, one process per GPU, native RCCL communicator (bucketed
    all-reduce, enqueued directly or — graphs — captured with the multi-step batch in a
    hipGraph and replayed): every rank verifies its results; the record is the metric's
    config, N = 1e9 in total split over the G GPUs; the ranks met over xGMI P2P; the
    untimed diagnostic batch says where the step's time went."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
              f"--nproc-per-node={g}", "--master-addr", "127.0.0.1", "--master-port",
              str(_port()), os.path.join(REPO, "bench.py"), "--gpus", str(g), "--steps", "48",
              "--warmup", "8"] + (["--graph-batches"] if graphs else []))
    assert p.returncode == 0, p.stderr[-3000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["verified"] and js["n_gpus"] == g and js["config"]["N"] == 10**9
    assert js["scaling"] == "strong" and js["config"]["n_per_gpu"] == 10**9 // g
    assert abs(js["abs_err"] - 1e-9) < 1e-13  # the N = 1e9 left-rule truncation
    assert js["config"]["bucketed_allreduce"] and js["config"]["multistep"]
    assert js["config"]["batch_launch"] == ("graph" if graphs else "direct")
    assert js["config"]["graphs"] == graphs and js["native_comm_verified"]
    d = js["diagnostic_batch"]
    assert d["path"] == "native" and d["allreduce_us"]["max"] > 0
    assert d["comm"]["allreduce_8b_us"] > 0 and d["comm"]["allgather_busbw_gbs"] > 0
    assert js["rccl_transport"].startswith("P2P") and js["rccl_nnodes"] == 1
    assert js["transport_verified"] and js["transport_error"] is None
    assert js["weak_1e9_per_gpu"]["N"] == g * 10**9 and js["weak_1e9_per_gpu"]["verified"]


@pytest.mark.parametrize("g", [2, 8])
def test_trainscan_threads_match_single(native, cuda, g):
    """The distributed train scan (allgather of {T1, T2, count}, rank carries) over G GPUs
    prints the single-GPU distance."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    one = _run([os.path.join(BIN, "trainscan"), "--json"])
    many = _run([os.path.join(BIN, "trainscan"), "--json", "--gpus", str(g)])
    assert one.returncode == 0 and many.returncode == 0, many.stderr[-2000:]
    a = json.loads(one.stdout.strip().splitlines()[-1])
    b = json.loads(many.stdout.strip().splitlines()[-1])
    _xgmi(b, g)
    assert b["distance"] == pytest.approx(a["distance"], rel=1e-13)
    assert b["sum_of_sums"] == pytest.approx(a["sum_of_sums"], rel=1e-12)


@pytest.mark.parametrize("g", [2, 8])
def test_bench_self_spawned_ranks(native, cuda, g):
    """`python bench.py --gpus G` without torchrun: the parent spawns G rank processes; RCCL
    reports G ranks; per-rank timings for all of them; BASELINE #3 strong point included."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    p = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(g), "--steps", "48",
              "--warmup", "8"])
    assert p.returncode == 0, p.stderr[-3000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["verified"] and js["n_gpus"] == g and js["launcher"] == "spawn"
    assert js["rccl_world"] == g and len(js["per_rank_ms"]) == g
    assert js["baseline3_strong_1e10"]["n_per_gpu"] == 10**10 // g
    assert js["config"]["N"] == 10**9 and js["rccl_transport"].startswith("P2P")
    assert js["rccl_nnodes"] == 1 and js["transport_verified"]


@pytest.mark.parametrize("g", [1, 2, 8])
def test_miintrun_gpu_ranks(native, cuda, slice_tol, g):
    """`miintrun -np G riemann` (the mpirun form): one process per GPU, RCCL bootstrapped from
    the launcher's environment (the native TCP rendezvous), rank 0 prints the global value —
    equal to the one-process integration. G = 1 runs on the one-GPU pool."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    run = os.path.join(BIN, "miintrun")
    if not os.path.exists(run):
        pytest.skip("miintrun not built")
    args = [os.path.join(BIN, "riemann"), "--integrand", "pi4", "--rule", "mid", "--json"]
    one = _run(args)
    many = _run([run, "-np", str(g), *args])
    assert one.returncode == 0 and many.returncode == 0, many.stderr[-2000:]
    a = json.loads(one.stdout.strip().splitlines()[-1])["result"]
    b = json.loads(many.stdout.strip().splitlines()[-1])
    assert b["gpus"] == g
    if g > 1:
        _xgmi(b, g)
    assert b["result"] == pytest.approx(a, rel=slice_tol(g) if g > 1 else 0, abs=0)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_cintegrate_gpus_match_single(native, cuda, g):
    """cintegrate --gpus G (the reference's CUDA program, cintegrate.cu:101-150, with its
    sample range split over G GPUs and the partials all-reduced): the 1-GPU value to 1e-13."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    one = _rec(_run([os.path.join(BIN, "cintegrate"), "--json"]))
    many = _rec(_run([os.path.join(BIN, "cintegrate"), "--json", "--gpus", str(g)]))
    _xgmi(many, g)
    assert many["result"] == pytest.approx(one["result"], rel=1e-13, abs=0)
    assert abs(many["result"] - 122000.004) < 1e-6


@pytest.mark.parametrize("g", [2, 8])
def test_table2d_gpus_match_single_and_oracle(native, cuda, g):
    """miint table2d --gpus G (BASELINE #5: the 4096^2 field's sample rows split over G GPUs,
    one RCCL all-reduce per graph batch): the 1-GPU value and the midpoint oracle."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    args = [os.path.join(BIN, "miint"), "table2d", "--grid", "4096", "--iters", "64"]
    one = _rec(_run(args))
    many = _rec(_run(args + ["--gpus", str(g)]))
    _xgmi(many, g)
    assert many["result"] == pytest.approx(one["result"], rel=1e-13, abs=0)
    assert many["rel_err_vs_oracle"] < 1e-12


@pytest.mark.parametrize("p", [3, 8])
def test_riemann_parity_master_worker_on_distinct_gpus(native, cuda, p):
    """riemann --parity as P processes on P GPUs (riemann.cpp:62-86): rank 0 coordinates,
    ranks 1..P-1 integrate worker slices on their own GPUs, rank 0 adds the gathered
    partials in rank order (bitwise), within 1e-10 of the host emulation of the reference."""
    if _devices() < p:
        pytest.skip(f"needs {p} HIP devices")
    n = 10**8
    r = _rec(_run(_np(p, os.path.join(BIN, "riemann"), "--parity", "--n", str(n), "--json")))
    _xgmi(r, p)
    W = p - 1
    assert r["parity"] and r["gpus"] == p and r["workers"] == W
    assert r["samples"] == W * (n // W)
    parts = r["partials"]
    assert len(parts) == p and parts[0] == 0.0
    acc = 0.0
    for q in range(1, p):  # the MPI_Recv loop's order and rounding
        acc += parts[q]
    assert acc == r["result"]
    host = _rec(_run([os.path.join(BIN, "riemann"), "--device", "cpu", "--parity", "--ranks",
                      str(p), "--n", str(n), "--json"]))
    assert abs(r["result"] - host["result"]) < 1e-10


@pytest.mark.parametrize("g", [2, 8])
def test_trainscan_replicate_every_rank_holds_the_table(native, cuda, g):
    """trainscan --replicate (4main.c:157: every rank ends with the whole 18 M-element table;
    here one RCCL allgather of 144 MB over xGMI): every rank's copy is bitwise the same
    (gathered FNV hashes), and it matches the 1-GPU table within roundoff."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    one = _rec(_run([os.path.join(BIN, "trainscan"), "--replicate", "--json"]))
    many = _rec(_run([os.path.join(BIN, "trainscan"), "--replicate", "--json", "--gpus", str(g)]))
    _xgmi(many, g)
    assert many["replicate"] and many["replicas_identical"] is True
    assert many["replica_n"] == one["replica_n"] == 18_000_000
    assert many["replica_sum"] == pytest.approx(one["replica_sum"], rel=1e-12)
    for x, y in zip(many["replica_at"], one["replica_at"]):
        assert x == pytest.approx(y, rel=1e-12, abs=1e-9)


@pytest.mark.parametrize("g", [2, 8])
def test_miint_comm_bandwidth_over_xgmi(native, cuda, g):
    """miint comm --gpus G: the 144 MB allgather (4main.c:157's table) runs over P2P with a
    nonzero bus bandwidth; the 8 B all-reduce (riemann.cpp:76's payload) has a latency."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    p = _run([os.path.join(BIN, "miint"), "comm", "--gpus", str(g), "--max-bytes", "144e6",
              "--iters", "5"])
    assert p.returncode == 0, p.stderr[-3000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    big = [r for r in rows if r["op"] == "allgather" and r["bytes"] / g >= 144e6 * 0.99]
    small = [r for r in rows if r["op"] == "allreduce" and r["bytes"] == 8]
    assert big and small
    for r in rows:
        assert r["gpus"] == g and r["rccl_transport"].startswith("P2P")
        assert r["rccl_nnodes"] == 1 and r["transport_verified"] is True
    assert big[0]["busbw_GBps"] > 1.0 and small[0]["us"] > 0
