"""CPU tests: generated velocity profile, oracle values, stdout formats."""
from __future__ import annotations

import math

import numpy as np
import pytest

from cuda_v_mpi_amd.utils import fixtures, oracle, output


def test_profile_shape_and_phases():
    v = fixtures.profile_table()
    assert v.shape == (1801,)
    assert v[0] == 0.0
    a = np.diff(v)
    # 7 phases: +jerk, hold, -jerk, cruise, -jerk, hold, +jerk (ex4vel.h)
    assert a[99] == pytest.approx(0.2904762, abs=1e-12)
    assert np.allclose(a[100:300], 0.2904762, atol=1e-12)
    assert np.allclose(a[399:1400], 0.0, atol=1e-12)
    assert v[400] == pytest.approx(87.14286, abs=1e-9)
    assert np.allclose(a[1499:1700], -0.2904762, atol=1e-12)
    assert abs(v[1800]) < 1e-12


def test_profile_bits_pinned():
    """The data table is bit-exact everywhere (also on the GPU box, where the reference
    is not mounted): its sha256 is pinned."""
    assert fixtures.profile_sha256(fixtures.profile_table()) == fixtures.PROFILE_SHA256


def test_profile_equals_reference_header_when_present():
    ref = fixtures.load_reference_table()
    if ref is None:
        pytest.skip("reference ex4vel.h not mounted")
    assert np.array_equal(ref, fixtures.profile_table())  # max |ref - data| == 0
    assert fixtures.profile_sha256(ref) == fixtures.PROFILE_SHA256


def test_generated_profile_reproduces_the_data():
    """The 7-phase jerk definition rebuilds the table to the spreadsheet's rounding noise."""
    gen, data = fixtures.generated_profile_table(), fixtures.profile_table()
    assert gen.shape == data.shape
    assert np.max(np.abs(gen - data)) < 2e-13


def test_native_profile_equals_python(native):
    assert np.array_equal(np.array(native.oracle.profile_table()), fixtures.profile_table())
    assert np.array_equal(np.array(native.oracle.generated_profile_table()),
                          fixtures.generated_profile_table())


def test_profile_exact_integral(native):
    assert fixtures.table_integral() == pytest.approx(122000.004, abs=1e-6)
    assert native.oracle.profile_exact_integral() == pytest.approx(122000.004, abs=1e-6)


@pytest.mark.parametrize("sp,sm,want", [(32, 2, 121999.800663), (30, 2, 122000.004000),
                                        (32, 3, 121823.051337)])
def test_cintegrate_parity(native, sp, sm, want):
    assert "%f" % native.oracle.cintegrate_parity(sp, sm) == "%f" % want
    assert oracle.cintegrate_parity(sp, sm) == pytest.approx(want, abs=2e-6)


@pytest.mark.parametrize("p,want", [(1, 122000.004030), (7, 0.0), (16, 117642.707174)])
def test_trainscan_parity(native, p, want):
    d, _ = native.oracle.trainscan_parity(p)
    assert "%f" % d == "%f" % want


@pytest.mark.parametrize("p", [2, 3, 4, 5, 6, 8, 9, 10])
def test_trainscan_parity_good_sizes(native, p):
    d, _ = native.oracle.trainscan_parity(p)
    assert 122000.003990 <= d <= 122000.004010


def test_trainscan_parity_python_twin(native):
    d_py, s_py = oracle.trainscan_parity(16)
    d_c, s_c = native.oracle.trainscan_parity(16)
    assert d_py == pytest.approx(d_c, abs=1e-6)
    assert s_py == pytest.approx(s_c, rel=1e-10)  # pairwise vs sequential summation


def test_phase2_sum_of_sums(native):
    _, s = native.oracle.trainscan_parity(1)
    assert s / 1e8 == pytest.approx(109861003.621919, abs=1e-3)


def test_riemann_mpi_parity(native):
    assert native.oracle.riemann_mpi_parity(1, 1e6) == 0.0          # B10: no workers
    assert native.oracle.riemann_mpi_parity(8, 1e6) == pytest.approx(2.0, abs=1e-10)
    assert oracle.riemann_mpi_parity(8, 1e6) == pytest.approx(
        native.oracle.riemann_mpi_parity(8, 1e6), abs=1e-12)


def test_analytic_values(native):
    I = native.Integrand
    assert native.oracle.analytic(I.pi4, 0, 1) == pytest.approx(math.pi, abs=1e-15)
    assert native.oracle.analytic(I.sin, 0, math.pi) == pytest.approx(2.0, abs=1e-15)
    d = native.oracle.analytic(I.train, 0, 1800, [], native.oracle.TRAIN_TS, native.oracle.TRAIN_VS)
    assert d == pytest.approx(121999.99983, abs=1e-4)
    assert native.oracle.analytic(I.table, 0, 1800) == pytest.approx(122000.004, abs=1e-6)


def test_serial_left_riemann_pi4_error(native):
    v = native.oracle.riemann_serial(native.Integrand.pi4, 0, 1, 10**6, native.Rule.left)
    assert v - math.pi == pytest.approx(1e-6, rel=1e-3)  # left-rule truncation is exactly h


def test_stdout_formats():
    assert output.fmt_seconds(1.325012) == "1.325012 seconds"
    assert output.fmt_cintegrate_distance(121999.800663) == "final distance is:121999.800663"
    assert (output.fmt_riemann_result(math.pi, 1e9, 2.0000000000002)
            == "The integral of f(x) from 0.0 to 3.14159265358979 with 1000000000 steps is "
               "2.0000000000002")
    assert output.fmt_step_size(10000) == "Step size of 10000"
    assert output.fmt_total_distance(122000.00403) == "Total distance traveled = 122000.004030"
