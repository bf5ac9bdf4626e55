"""Runtime integrands (miint/expr.hpp) on the CPU: the generated kernel source, the hipRTC
compile for gfx950 (no device needed) and the expression checks that run before anything is
compiled. The reference hard-wires its integrand (riemann.cpp:37) and recompiles to change
it; here the expression is compiled at run time. GPU numerics: tests/test_expr_gpu.py."""
from __future__ import annotations

import pytest


def test_expr_source_wraps_the_expression(native):
    src = native.expr_source("exp(-x*x)")
    assert "return (exp(-x*x));" in src
    assert "miint_expr_partials" in src and "miint_expr_finalize" in src


def test_expr_compiles_for_gfx950_without_a_device(native):
    code = native.expr_compile("sin(x) * exp(-0.5 * x * x) + pow(fabs(x), 1.5)")
    assert code[:4] == b"\x7fELF" or code[:4] == b"__CL"  # code object (or offload bundle)
    assert native.expr_compile("sin(x) * exp(-0.5 * x * x) + pow(fabs(x), 1.5)") == code


@pytest.mark.parametrize("bad", ["x; x", "x) { return 0", "asm(\"s_nop 0\")", "asm (x)",
                                 "__builtin_amdgcn_s_sleep(1)", "x\\", "#define y", "'a'",
                                 "", "x" * 5000,
                                 # digraphs: { } [ ] # spelled with allowed characters
                                 "x <% return 0; %>", "x <: 0 :>", "%:define y", "x%>",
                                 "(<%%>)"])
def test_expr_rejected_before_compiling(native, bad):
    with pytest.raises(RuntimeError, match="expression"):
        native.expr_source(bad)


def test_expr_compile_error_carries_the_log(native):
    with pytest.raises(RuntimeError, match="does not compile"):
        native.expr_compile("1.0 / (1.0 + y)")


# ------------------------------------------------------------------ host side (HostExpr)
import json  # noqa: E402
import math  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("expr,a,b,want", [
    ("exp(-x*x)", 0.0, 3.0, math.sqrt(math.pi) / 2 * math.erf(3.0)),
    ("4.0 / (1.0 + x * x)", 0.0, 1.0, math.pi),
    ("x > 1.0 ? 2.0 * x - 1.0 : x * x", 0.0, 2.0, 7.0 / 3.0),
])
def test_host_expr_midpoint_analytic(native, expr, a, b, want):
    """The expression compiled for the host cores (system compiler, dlopen), midpoint rule."""
    he = native.HostExpr(expr)
    v = he.integrate(a, b, 2_000_001, native.Rule.mid, 0, 2_000_001, native.HostPool(3))
    assert v == pytest.approx(want, rel=1e-10)


def test_host_expr_threads_slices_and_oracle(native):
    """sin(x) on [0, pi], left rule: the long-double oracle to 1e-14, 1 vs 5 threads to
    1e-15, rank slices summing to the whole."""
    from cuda_v_mpi_amd.parallel.decomposition import rank_slice

    n = 3_000_017
    he = native.HostExpr("sin(x)")
    v1 = he.integrate(0.0, math.pi, n, native.Rule.left, 0, n, native.HostPool(1))
    p5 = native.HostPool(5)
    v5 = he.integrate(0.0, math.pi, n, native.Rule.left, 0, n, p5)
    o = native.oracle.riemann_serial(native.Integrand.sin, 0.0, math.pi, n, native.Rule.left)
    assert v1 == pytest.approx(o, rel=1e-14) and v5 == pytest.approx(v1, rel=1e-15)
    parts = [he.integrate(0.0, math.pi, n, native.Rule.left, *rank_slice(n, r, 3), p5)
             for r in range(3)]
    assert math.fsum(parts) == pytest.approx(v5, rel=1e-15)


def test_host_expr_rejections(native):
    with pytest.raises(RuntimeError, match="not allowed"):
        native.HostExpr("x; system(0)")
    with pytest.raises(RuntimeError, match="does not compile"):
        native.HostExpr("1.0 / (1.0 + y)")
    with pytest.raises(RuntimeError, match="digraph"):  # a block smuggled past the filter
        native.HostExpr("x + (<%%>)")


def test_expr_modulo_and_comparisons_still_allowed(native):
    """The digraph rule leaves the operators it shares characters with: %, <, >, ?: ."""
    src = native.expr_source("x < 0.5 ? fmod(x, 0.25) : (x > 0.75 ? 1.0 : x * x)")
    assert "fmod(x, 0.25)" in src
    v = native.HostExpr("(x < 0.5) ? 2.0 : 0.0").integrate(0.0, 1.0, 1000,
                                                          native.Rule.mid, 0, 1000,
                                                          native.HostPool(1))
    assert v == pytest.approx(1.0, rel=1e-12)


def test_cli_and_compare_host_expr():
    exe = os.path.join(REPO, "build", "bin", "riemann")
    if not os.path.exists(exe):
        pytest.skip("CLI not built")
    p = subprocess.run([exe, "--device", "cpu", "--expr", "exp(-x*x)", "--a", "0", "--b", "3",
                        "--rule", "mid", "--n", "1e7", "--json"], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.splitlines()[-1])
    assert rec["result"] == pytest.approx(math.sqrt(math.pi) / 2 * math.erf(3.0), rel=1e-12)
    c = subprocess.run([sys.executable, "-m", "cuda_v_mpi_amd", "compare", "--expr", "exp(-x*x)",
                        "--a", "0", "--b", "3", "--n", "1e7", "--reps", "1", "--rule", "mid"],
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert c.returncode == 0, c.stderr
    rows = [json.loads(x) for x in c.stdout.splitlines()]
    host = next(r for r in rows if r.get("side") == "host")
    assert host["value"] == pytest.approx(rec["result"], rel=1e-14)


def test_integrate_expr_host_api(native):
    from cuda_v_mpi_amd import integrate_expr

    want = math.sqrt(math.pi) / 2 * math.erf(3.0)
    r = integrate_expr("exp(-x*x)", 0.0, 3.0, n=10**6, rule="mid", backend="host", threads=2,
                       analytic=want)
    assert r.abs_err < 1e-12 and r.integrand == "expr:exp(-x*x)" and r.seconds_device > 0
    with pytest.raises(ValueError):
        integrate_expr("x", 0, 1, backend="cpu")
