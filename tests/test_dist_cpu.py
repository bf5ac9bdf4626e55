"""Multi-process tests of the decomposition + collective path on CPU (gloo, world_size 2-4).

The reference's distributed programs need `mpirun` and real nodes ("multi-node
without a cluster: nothing is provided"). Here the same decomposition code that the GPU
path uses is exercised by real torch.distributed processes on the CPU backend.
"""
from __future__ import annotations

import math
import os

import pytest
import torch.multiprocessing as mp

from cuda_v_mpi_amd.parallel import decomposition


def _free_port() -> int:
    from bench import rendezvous_port  # below the ephemeral range (no self-connect)

    return rendezvous_port()


def _worker(rank: int, world: int, port: int, name: str, n: int, rule: str, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cuda_v_mpi_amd import Integrator
    from cuda_v_mpi_amd.parallel import dist as mdist

    ctx = mdist.init(backend="gloo")
    try:
        r = Integrator(name, n=n, rule=rule, backend="cpu", ctx=ctx).run()
        gathered = ctx.all_gather_scalars(float(ctx.rank))
        q.put((rank, r.value, gathered))
    finally:
        ctx.destroy()


def _run_world(world: int, name: str, n: int, rule: str = "left"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, n, rule, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_cpu_riemann_matches_single(world):
    from cuda_v_mpi_amd import Integrator

    n = 1_000_003  # not divisible by world: remainder samples must not be dropped
    single = Integrator("pi4", n=n, backend="cpu").run().value
    res = _run_world(world, "pi4", n)
    for rank, value, gathered in res:
        assert value == pytest.approx(single, rel=1e-13)      # every rank holds the total
        assert gathered == [float(r) for r in range(world)]
    assert abs(res[0][1] - math.pi - 1.0 / n) < 1e-9


def test_distributed_cpu_sin_mid():
    res = _run_world(2, "sin", 400_000, rule="mid")
    assert res[0][1] == pytest.approx(2.0, abs=1e-11)


# ------------------------------------------------------------------ pure decomposition
@pytest.mark.parametrize("n,world", [(10, 3), (10**9, 8), (7, 8), (2**40 + 3, 7)])
def test_rank_slice_covers_exactly(n, world):
    spans = [decomposition.rank_slice(n, r, world) for r in range(world)]
    pos = 0
    for b, c in spans:
        assert b == pos
        pos += c
    assert pos == n
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_master_worker_partition_is_reference():
    # riemann.cpp:65-73: P ranks -> P-1 workers; P=1 has none (prints 0)
    assert decomposition.master_worker_slices(1, 1e9) == []
    sl = decomposition.master_worker_slices(8, 1e9)
    assert len(sl) == 7 and sl[0][0] == 0.0 and sl[-1][1] == pytest.approx(math.pi)
    assert all(c == int(1e9 / 7) for _, _, c in sl)


def test_trainscan_partitions_mismatch_when_p_does_not_divide_1800():
    # 4main.c:76-78 vs 90-91: fill by seconds, scan by elements
    p7 = decomposition.trainscan_partitions(7)
    assert p7[-1][1] == 1799 * 10000         # last second never filled
    assert p7[-1][3] == 7 * (18_000_000 // 7) < 18_000_000  # residual never scanned
    p8 = decomposition.trainscan_partitions(8)
    assert all(f0 == s0 and f1 == s1 for f0, f1, s0, s1 in p8[:1])


def test_cintegrate_coverage():
    assert decomposition.coverage_seconds(64) == 1792   # 8 s dropped
    assert decomposition.coverage_seconds(60) == 1800
    ch = decomposition.cintegrate_chunks(32, 2)
    assert ch[1][0] - ch[0][0] == 280_000


def test_torchrun_table2d_cpu_rows_split_over_ranks():
    """`python -m cuda_v_mpi_amd table2d` under torchrun (3 gloo ranks on the CPU): each rank
    integrates its row slice (rows not divisible by 3) and the all-reduced sum is the whole
    field's midpoint sum."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=3", "--master-addr", "127.0.0.1",
                        f"--master-port={_free_port()}", "-m", "cuda_v_mpi_amd", "table2d",
                        "--backend", "cpu", "--grid", "301"],
                       cwd=repo, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=repo))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 1 and rows[0]["gpus"] == 3  # rank 0 prints
    assert rows[0]["rel_err_vs_oracle"] < 1e-13


def test_shared_device_rccl_env(monkeypatch):
    """MIINT_OVERSUBSCRIBE=1 (ranks share a GPU): each rank a host of its own to RCCL, socket
    transport on loopback; without it nothing is touched."""
    from cuda_v_mpi_amd.parallel import dist as mdist

    for k in ("MIINT_OVERSUBSCRIBE", "NCCL_HOSTID", "NCCL_SOCKET_IFNAME", "NCCL_IB_DISABLE"):
        monkeypatch.delenv(k, raising=False)
    mdist.prepare_shared_device_rccl(3)
    assert not mdist.ranks_share_devices() and "NCCL_HOSTID" not in os.environ
    monkeypatch.setenv("MIINT_OVERSUBSCRIBE", "1")
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "eth9")  # a user's choice is kept
    mdist.prepare_shared_device_rccl(3)
    assert mdist.ranks_share_devices()
    assert os.environ["NCCL_HOSTID"] == "miint-shared-rank-3"
    assert os.environ["NCCL_SOCKET_IFNAME"] == "eth9" and os.environ["NCCL_IB_DISABLE"] == "1"
