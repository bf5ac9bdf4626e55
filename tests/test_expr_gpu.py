"""Runtime integrands on the MI355X: f(x) as an expression, compiled with hipRTC for gfx950
(csrc/runtime/expr.cpp), against the built-in kernels, the long-double oracle and analytic
values; rank slices, a communicator, determinism and the CLI."""
from __future__ import annotations

import json
import math
import os
import subprocess

import pytest

from cuda_v_mpi_amd.ops import kernels
from cuda_v_mpi_amd.parallel import loopback

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_expr_sin_equals_oracle_and_builtin(native, cuda):
    """sin(x) on [0, pi], left rule, N = 1e7: the long-double serial oracle to 1e-14 and the
    built-in Sin kernel (a different per-sample algorithm) to 1e-14."""
    from cuda_v_mpi_amd import Integrator

    n = 10**7
    v = kernels.riemann_expr("sin(x)", 0.0, math.pi, n)
    o = native.oracle.riemann_serial(native.Integrand.sin, 0.0, math.pi, n, native.Rule.left)
    assert v == pytest.approx(o, rel=1e-14)
    assert v == pytest.approx(Integrator("sin", n=n).run().value, rel=1e-14)


def test_expr_pi4_headline_config(native, cuda):
    """The headline integrand written as an expression, N = 1e9 left rule: |err| = h."""
    v = kernels.riemann_expr("4.0 / (1.0 + x * x)", 0.0, 1.0, 10**9)
    assert abs(v - math.pi - 1e-9) < 1e-15


@pytest.mark.parametrize("expr,a,b,want", [
    ("exp(-x*x)", 0.0, 3.0, math.sqrt(math.pi) / 2 * math.erf(3.0)),
    ("1.0 / sqrt(1.0 - x*x)", -0.5, 0.5, 2 * math.asin(0.5)),
    ("x > 1.0 ? 2.0 * x - 1.0 : x * x", 0.0, 2.0, 7.0 / 3.0),
    ("pow(x, 3.0) - 2.0 * x", -1.0, 3.0, (81 - 1) / 4 - (9 - 1)),
])
def test_expr_midpoint_analytic(cuda, expr, a, b, want):
    v = kernels.riemann_expr(expr, a, b, 4_000_001, rule="mid")
    assert v == pytest.approx(want, rel=1e-9, abs=1e-10)


def test_expr_slices_and_determinism(native, cuda):
    """Four rank slices of one rule sum to the whole; a second run is bitwise equal."""
    from cuda_v_mpi_amd.parallel.decomposition import rank_slice

    n = 12_345_679
    whole = kernels.riemann_expr("cos(3.0 * x) * x", 0.0, 2.0, n)
    assert kernels.riemann_expr("cos(3.0 * x) * x", 0.0, 2.0, n) == whole
    parts = [kernels.riemann_expr("cos(3.0 * x) * x", 0.0, 2.0, n, i_begin=b, n_local=c)
             for b, c in (rank_slice(n, r, 4) for r in range(4))]
    assert math.fsum(parts) == pytest.approx(whole, rel=1e-14)


def test_expr_with_a_communicator(native, cuda):
    """Three loopback ranks: each integrates its slice, the communicator all-reduces, every
    rank holds the one-rank value."""
    from cuda_v_mpi_amd.parallel.decomposition import rank_slice

    n = 3_000_001
    one = kernels.riemann_expr("atan(x)", 0.0, 5.0, n)

    def body(rank, comm):
        ei = native.ExprIntegrator("atan(x)", 0)
        b, c = rank_slice(n, rank, 3)
        return ei.integrate(0.0, 5.0, n, native.Rule.left, b, c, 1.0, comm)
    out = loopback.run_ranks(3, body)
    for v in out:
        assert v == pytest.approx(one, rel=1e-14)
        assert v == out[0]


def test_cli_riemann_expr(cuda):
    exe = os.path.join(REPO, "build", "bin", "riemann")
    if not os.path.exists(exe):
        pytest.skip("CLI not built")
    p = subprocess.run([exe, "--expr", "exp(-x*x)", "--a", "0", "--b", "3", "--n", "1e8",
                        "--rule", "mid", "--analytic", repr(math.sqrt(math.pi) / 2 * math.erf(3)),
                        "--json", "--iters", "5"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert lines[1].startswith("The integral of f(x) from 0.0 to 3 with 100000000 steps is 0.8862")
    rec = json.loads(lines[-1])
    assert rec["abs_err"] < 1e-13 and rec["subintervals_per_s"] > 1e10


def test_compare_expr_gpu_and_host(native, cuda):
    """`compare --expr`: the same expression compiled for gfx950 (hipRTC) and for the host
    cores agrees to 1e-12; the GPU row is the faster one."""
    p = subprocess.run(["python", "-m", "cuda_v_mpi_amd", "compare", "--expr", "exp(-x*x)",
                        "--a", "0", "--b", "3", "--n", "1e8", "--rule", "mid", "--reps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert p.returncode == 0, p.stderr
    rows = [json.loads(x) for x in p.stdout.splitlines()]
    by = {r["side"]: r for r in rows if "side" in r}
    assert by["gpu"]["value"] == pytest.approx(by["host"]["value"], rel=1e-12)
    assert by["gpu"]["value"] == pytest.approx(math.sqrt(math.pi) / 2 * math.erf(3.0), rel=1e-12)
    assert rows[-1]["speedup_gpu_vs_host"] > 1.0


def test_integrate_expr_hip_api(cuda):
    from cuda_v_mpi_amd import integrate_expr

    r = integrate_expr("4.0 / (1.0 + x * x)", 0.0, 1.0, n=10**8, rule="mid", analytic=math.pi)
    assert r.abs_err < 1e-14
