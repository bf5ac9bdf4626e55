"""Multi-GPU tests (SURVEY §7.4 "Comm tests ... 2/4/8 when available"): run only where the
box shows at least that many HIP devices, and compare with the single-GPU result.

The gpurun pool gives one GPU: there these skip, and the 1-rank RCCL graph path
(tests/test_gpu_runtime.py::test_plan_rccl_stage_on_one_gpu) plus the gloo tests carry the
multi-rank logic. RCCL refuses two ranks on one device (tools/two_rank_native_probe.py).
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


@pytest.mark.parametrize("g", [2, 4, 8])
def test_cli_threads_ncclcomminitall(native, cuda, g):
    """One process driving G GPUs (ncclCommInitAll + threads): the global sum of the G
    rank slices equals the 1-GPU integration of the same N to fp64 roundoff."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    one = _run([os.path.join(BIN, "riemann"), "--integrand", "pi4", "--rule", "mid", "--json"])
    many = _run([os.path.join(BIN, "riemann"), "--integrand", "pi4", "--rule", "mid", "--json",
                 "--gpus", str(g)])
    assert one.returncode == 0 and many.returncode == 0, many.stderr[-2000:]
    a = json.loads(one.stdout.strip().splitlines()[-1])["result"]
    b = json.loads(many.stdout.strip().splitlines()[-1])["result"]
    assert b == pytest.approx(a, rel=1e-15, abs=0)


@pytest.mark.parametrize("g", [2, 8])
def test_bench_torchrun_rccl(native, cuda, g):
    """bench.py under torchrun, one process per GPU, native RCCL communicator in the step
    graph (bucketed all-reduce): every rank verifies its results; weak scaling grows N."""
    if _devices() < g:
        pytest.skip(f"needs {g} HIP devices")
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
              f"--nproc-per-node={g}", "--master-addr", "127.0.0.1", "--master-port",
              str(_port()), os.path.join(REPO, "bench.py"), "--gpus", str(g), "--steps", "48",
              "--warmup", "8"])
    assert p.returncode == 0, p.stderr[-3000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["verified"] and js["n_gpus"] == g and js["config"]["N"] == g * 10**9
    assert js["config"]["bucketed_allreduce"] and js["config"]["graphs"]


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


@pytest.mark.parametrize("g", [1, 2, 8])
def test_miintrun_gpu_ranks(native, cuda, g):
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
    assert b["result"] == pytest.approx(a, rel=1e-15, abs=0)
