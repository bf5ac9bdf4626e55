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
                                 "", "x" * 5000])
def test_expr_rejected_before_compiling(native, bad):
    with pytest.raises(RuntimeError, match="expression"):
        native.expr_source(bad)


def test_expr_compile_error_carries_the_log(native):
    with pytest.raises(RuntimeError, match="does not compile"):
        native.expr_compile("1.0 / (1.0 + y)")
