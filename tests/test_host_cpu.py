"""The host engine (miint/host.hpp): the reference's own CPU/MPI side, native, on the CPU.

riemann.cpp and 4main.c are CPU programs: P processes running scalar
loops and gathering by MPI point-to-point. These tests pin the host engine that replaces them
(vector threads, rank-order host collectives over TCP, the threaded train scan) against the
long-double oracles, against each other across thread counts, ISAs and ranks, and against
the reference's printed values. No GPU is touched.
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys

import pytest

from cuda_v_mpi_amd.models import integrands

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
INTEGRANDS = ["pi4", "sin", "poly", "train", "table"]


def _cfg(native, name, n, rule="mid"):
    spec = integrands.get(name)
    c = native.RiemannConfig()
    c.integrand = getattr(native.Integrand, spec.name)
    c.a, c.b, c.n = spec.a, spec.b, int(n)
    c.rule = getattr(native.Rule, rule)
    c.coef = list(spec.coef)
    c.p0, c.p1 = spec.p0, spec.p1
    c.table = spec.native_table()
    return c, spec


@pytest.mark.parametrize("name", INTEGRANDS)
@pytest.mark.parametrize("rule", ["left", "mid"])
def test_host_riemann_matches_long_double_oracle(native, name, rule):
    """Per-sample fp64 on vector threads vs the long-double Kahan serial sum, N = 1e6."""
    c, spec = _cfg(native, name, 10**6, rule)
    v = native.host_riemann(c, 0, c.n, native.HostPool(4))
    o = native.oracle.riemann_serial(c.integrand, c.a, c.b, c.n, c.rule, list(spec.coef),
                                     spec.p0, spec.p1)
    assert v == pytest.approx(o, rel=2e-15, abs=1e-15)


@pytest.mark.parametrize("name", INTEGRANDS)
def test_host_riemann_threads_and_determinism(native, name):
    """1, 3 and 8 threads (odd N, uneven thread slices, vector tails) agree to 1e-15; a
    fixed thread count is bitwise reproducible."""
    c, _ = _cfg(native, name, 3_000_001)
    vals = {t: native.host_riemann(c, 0, c.n, native.HostPool(t)) for t in (1, 3, 8)}
    for v in vals.values():
        assert v == pytest.approx(vals[1], rel=1e-15)
    p3 = native.HostPool(3)
    assert native.host_riemann(c, 0, c.n, p3) == native.host_riemann(c, 0, c.n, p3)


def test_host_riemann_rank_slices_tile_the_rule(native):
    """Four ranks' slices of one rule (the exact 64-bit rank_slice cover) sum to the whole;
    N = 5e9 > 2^32 exercises the 64-bit index (riemann.cpp's int counter overflows, B9)."""
    from cuda_v_mpi_amd.parallel.decomposition import rank_slice

    pool = native.HostPool(0)
    c, _ = _cfg(native, "pi4", 10**7)
    whole = native.host_riemann(c, 0, c.n, pool)
    parts = [native.host_riemann(c, *rank_slice(c.n, r, 4), pool) for r in range(4)]
    assert math.fsum(parts) == pytest.approx(whole, rel=1e-15)
    c, spec = _cfg(native, "pi4", 5 * 10**9, "mid")
    b, n = rank_slice(c.n, 3, 4)  # the last quarter only: indices above 2^32
    v = native.host_riemann(c, b, n, pool)
    assert v == pytest.approx(4 * (math.atan(1.0) - math.atan(0.75)), rel=1e-13)


def test_host_riemann_rejects_bad_slices(native):
    c, _ = _cfg(native, "pi4", 1000)
    with pytest.raises(RuntimeError, match="outside"):
        native.host_riemann(c, 900, 200, native.HostPool(2))


@pytest.mark.parametrize("isa", ["avx2", "base"])
def test_host_isa_builds_agree(native, isa):
    """The AVX2 and baseline builds of the kernels give the AVX-512 build's values (all use
    true fma); MIINT_HOST_ISA caps the dispatch in a fresh process."""
    code = ("import json, sys; sys.path.insert(0, %r)\n"
            "from cuda_v_mpi_amd import native\n"
            "from tests.test_host_cpu import _cfg\n"
            "m = native(); out = {'isa': m.host_isa()}\n"
            "for f in %r:\n"
            "    c, _ = _cfg(m, f, 200_003)\n"
            "    out[f] = m.host_riemann(c, 0, c.n, m.HostPool(2))\n"
            "print(json.dumps(out))\n") % (REPO, INTEGRANDS)
    env = dict(os.environ, MIINT_HOST_ISA=isa)
    got = json.loads(subprocess.run([sys.executable, "-c", code], env=env, cwd=REPO,
                                    capture_output=True, text=True, check=True).stdout)
    if native.host_isa() == "base" or (isa == "avx2" and native.host_isa() == "avx2"):
        pytest.skip("this CPU has nothing above the requested ISA")
    assert got["isa"] == isa
    p2 = native.HostPool(2)
    for f in INTEGRANDS:
        c, _ = _cfg(native, f, 200_003)
        assert got[f] == pytest.approx(native.host_riemann(c, 0, c.n, p2), rel=1e-15), f


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_host_mpi_parity_bitwise_equals_oracle(native, P):
    """riemann.cpp's master/worker program on threads is bitwise the serial emulation
    (P = 1 -> 0 workers -> 0)."""
    got = native.host_riemann_mpi_parity(P, 1e6, math.pi, native.HostPool(3))
    assert got == native.oracle.riemann_mpi_parity(P, 1e6)
    if P == 1:
        assert got == 0.0


def test_host_trainscan_totals(native):
    """distance = the exact knot-sampled integral 122000.004 (the reference's sequential sums
    drift to ...004030); sum of sums consistent across 1 and 8 threads and with the kept
    arrays' last elements (compensated running sums)."""
    one = native.host_trainscan(10000, 1800, native.HostPool(1), None, False)
    eight = native.host_trainscan(10000, 1800, native.HostPool(8), None, True)
    assert one["distance"] == pytest.approx(122000.004, rel=1e-14)
    assert eight["distance"] == pytest.approx(one["distance"], rel=1e-15)
    assert eight["sum_of_sums"] == pytest.approx(one["sum_of_sums"], rel=1e-14)
    # the 4main.c phase-2 value (its own drifting sums print 109861003.621919)
    assert one["sum_of_sums"] / 1e8 == pytest.approx(109861003.621919, rel=1e-9)
    vel, pos = eight["velocity"], eight["position"]
    assert len(vel) == len(pos) == 18_000_000
    assert vel[-1] / 1e4 == pytest.approx(eight["distance"], rel=1e-14)
    assert pos[-1] == pytest.approx(eight["sum_of_sums"], rel=1e-14)


def test_host_trainscan_prefix_matches_fsum(native):
    """The first 20 001 running sums against exact (fsum) prefixes of the same samples."""
    r = native.host_trainscan(10000, 3, native.HostPool(3), None, True)  # 30 000 samples
    tab = native.oracle.profile_table()
    v = []
    for i in range(20_001):
        s = min(int((i + 0.5) / 10000), len(tab) - 2)
        v.append(math.fma(tab[s + 1] - tab[s], (i - s * 10000) * 1e-4, tab[s])
                 if hasattr(math, "fma") else tab[s] + (tab[s + 1] - tab[s]) * ((i - s * 10000) * 1e-4))
    for k in (0, 1, 9_999, 10_000, 20_000):
        assert r["velocity"][k] == pytest.approx(math.fsum(v[:k + 1]), rel=1e-14)


def _free_port() -> int:
    from bench import rendezvous_port  # below the ephemeral range (no self-connect)

    return rendezvous_port()


_COMM_RANK = r"""
import json, sys
sys.path.insert(0, {repo!r})
from cuda_v_mpi_amd import native
m = native()
r, w, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
c = m.HostComm("127.0.0.1", port, r, w, 60.0)
out = {{}}
out["allreduce"] = c.allreduce_sum([0.1 * (r + 1), 1e16 if r == 0 else 1.0, -r])
out["allgather"] = c.allgather([r, 10.0 * r])
out["bcast"] = c.broadcast([float(r)] * 3, w - 1)
c.barrier()
pool = m.HostPool(2)
s = m.host_trainscan(10000, 60, pool, c, False)
out["scan"] = [s["distance"], s["sum_of_sums"], s["begin"], s["count"]]
print(json.dumps(out))
"""


def test_host_comm_collectives_and_ranked_trainscan(native):
    """4 host processes over the TCP star: rank-order sums (bitwise equal on every rank),
    allgather in rank order, broadcast from the last rank, barrier; the train scan across
    the 4 ranks equals the one-rank scan."""
    W, port = 4, _free_port()
    code = _COMM_RANK.format(repo=REPO)
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r), str(W), str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(W)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e
        outs.append(json.loads(o))
    want = [((0.1 * 1 + 0.1 * 2) + 0.1 * 3) + 0.1 * 4, ((1e16 + 1.0) + 1.0) + 1.0, -6.0]
    for r, o in enumerate(outs):
        assert o["allreduce"] == want
        assert o["allgather"] == [x for q in range(W) for x in (q, 10.0 * q)]
        assert o["bcast"] == [float(W - 1)] * 3
        assert o["scan"][:2] == outs[0]["scan"][:2]
    assert sum(o["scan"][3] for o in outs) == 600_000
    one = native.host_trainscan(10000, 60, native.HostPool(2), None, False)
    assert outs[0]["scan"][0] == pytest.approx(one["distance"], rel=1e-14)
    assert outs[0]["scan"][1] == pytest.approx(one["sum_of_sums"], rel=1e-13)


def test_host_comm_times_out_without_peers(native):
    with pytest.raises(RuntimeError, match="connected before the timeout"):
        native.HostComm("127.0.0.1", _free_port(), 0, 2, 0.5)


def _run(args, env=None):
    p = subprocess.run(args, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stderr
    return p.stdout


@pytest.fixture(scope="module")
def cli_bins():
    if not all(os.path.exists(os.path.join(BIN, b)) for b in ("riemann", "cintegrate", "trainscan")):
        pytest.skip("native CLIs not built (make cli)")
    return BIN


def test_cli_device_cpu_reference_lines(cli_bins):
    """--device cpu prints the reference's exact lines on a GPU-less box:
    `mpirun -np 8 ./riemann` -> 2.0000000000002 (its own numerics, P-1 workers), -np 1 -> 0,
    cintegrate 122000.004000 / parity 121999.800663, 4main P = 7 -> 0.000000 and
    P = 16 -> 117642.707174."""
    out = _run([os.path.join(BIN, "riemann"), "--device", "cpu", "--parity", "--ranks", "8"])
    assert out.splitlines()[1] == ("The integral of f(x) from 0.0 to 3.14159265358979 with "
                                   "1000000000 steps is 2.0000000000002")
    out = _run([os.path.join(BIN, "riemann"), "--device", "cpu", "--parity", "--ranks", "1"])
    assert out.splitlines()[1].endswith("steps is 0")
    assert _run([os.path.join(BIN, "cintegrate"), "--device", "cpu"]).splitlines()[1] == \
        "final distance is:122000.004000"
    assert _run([os.path.join(BIN, "cintegrate"), "--device", "cpu", "--parity"]).splitlines()[1] \
        == "final distance is:121999.800663"
    for P, want in ((7, "0.000000"), (16, "117642.707174"), (1, "122000.004030")):
        out = _run([os.path.join(BIN, "trainscan"), "--device", "cpu", "--parity", "--ranks", str(P)])
        assert out.splitlines()[0] == "Step size of 10000"
        assert out.splitlines()[2] == f"Total distance traveled = {want}"
    out = _run([os.path.join(BIN, "trainscan"), "--device", "cpu"])
    assert out.splitlines()[2] == "Total distance traveled = 122000.004000"


def test_cli_device_cpu_host_ranks(cli_bins):
    """riemann / trainscan --device cpu as 3 host processes (torchrun-style env): rank 0
    prints the one-process value (rank-order host all-reduce, carries over ranks)."""
    def ranks(cmd, W=3):
        port = _free_port()
        procs = []
        for r in range(W):
            env = dict(os.environ, WORLD_SIZE=str(W), RANK=str(r), LOCAL_RANK=str(r),
                       LOCAL_WORLD_SIZE=str(W), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=300) for p in procs]
        assert all(p.returncode == 0 for p in procs), [o[1] for o in outs]
        assert all(o[0] == "" for o in outs[1:])  # only rank 0 prints
        return json.loads(outs[0][0].splitlines()[-1])

    rie = [os.path.join(BIN, "riemann"), "--device", "cpu", "--integrand", "pi4", "--n", "1e8",
           "--rule", "mid", "--json"]
    multi, single = ranks(rie), json.loads(_run(rie).splitlines()[-1])
    assert multi["ranks"] == 3 and single["ranks"] == 1
    assert multi["result"] == pytest.approx(single["result"], rel=1e-15)
    assert multi["abs_err"] < 1e-14
    ts = [os.path.join(BIN, "trainscan"), "--device", "cpu", "--json"]
    multi = ranks(ts)
    assert multi["distance"] == pytest.approx(122000.004, rel=1e-14)


def test_python_host_backend_and_compare(native):
    from cuda_v_mpi_amd import Integrator

    r = Integrator("sin", n=10**7, backend="host", threads=3).run()
    assert abs(r.value - 2.0) < 1e-13 and r.seconds_device > 0
    p = subprocess.run([sys.executable, "-m", "cuda_v_mpi_amd", "compare", "--n", "2e7",
                        "--reps", "1"], capture_output=True, text=True, cwd=REPO, timeout=300)
    assert p.returncode == 0, p.stderr
    rows = [json.loads(x) for x in p.stdout.splitlines()]
    sides = {x.get("side") for x in rows}
    assert {"host", "reference-program", "gpu"} <= sides
    ref = next(x for x in rows if x.get("side") == "reference-program")
    assert ref["value"] == native.oracle.riemann_mpi_parity(8, 2e7)
