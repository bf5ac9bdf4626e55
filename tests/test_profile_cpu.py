"""User velocity profiles (`--profile FILE`): the reference's table was generated from a
spreadsheet CSV (ex4vel.h:1-5) and compiled in; here a profile of one's own is read at run
time (oracle::load_profile) and integrated by every tool. CPU side; GPU: test_profile_gpu.py.
"""
from __future__ import annotations

import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
TRIANGLE = [0.0, 10.0, 20.0, 30.0, 40.0, 30.0, 20.0, 10.0, 0.0]  # integral 160


@pytest.fixture
def tri_csv(tmp_path):
    p = tmp_path / "tri.csv"
    p.write_text("# a triangle, 1 s apart\n0, 10, 20, 30\n\n40;30\t20 10\n  # more\n0\n")
    return str(p)


def test_load_profile_and_exact_integral(native, tri_csv):
    v = native.oracle.load_profile(tri_csv)
    assert v == TRIANGLE
    assert native.oracle.table_integral(v, 0.0, 8.0) == 160.0
    assert native.oracle.table_integral(v, 1.5, 2.5) == pytest.approx(20.0)
    # the built-in profile's exact integral through the same function
    assert native.oracle.table_integral(native.oracle.profile_table(), 0.0, 1800.0) == \
        pytest.approx(native.oracle.profile_exact_integral(), rel=1e-15)


@pytest.mark.parametrize("text,msg", [("1, 2, x\n", "not a finite number"), ("5\n", "at least 2"),
                                       ("1, nan\n", "not a finite number")])
def test_load_profile_rejects(native, tmp_path, text, msg):
    p = tmp_path / "bad.csv"
    p.write_text(text)
    with pytest.raises(RuntimeError, match=msg):
        native.oracle.load_profile(str(p))
    with pytest.raises(RuntimeError, match="cannot read"):
        native.oracle.load_profile(str(tmp_path / "missing.csv"))


def test_host_trainscan_with_a_profile(native):
    r = native.host_trainscan(10000, 8, native.HostPool(3), None, True, TRIANGLE)
    assert r["distance"] == pytest.approx(160.0, rel=1e-14)
    assert len(r["velocity"]) == 80_000


def _run(args):
    p = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return p.stdout


def test_cli_profile_device_cpu(tri_csv):
    if not os.path.exists(os.path.join(BIN, "cintegrate")):
        pytest.skip("CLIs not built")
    assert _run([os.path.join(BIN, "cintegrate"), "--device", "cpu", "--profile", tri_csv]) \
        .splitlines()[1] == "final distance is:160.000000"
    out = _run([os.path.join(BIN, "trainscan"), "--device", "cpu", "--profile", tri_csv])
    assert out.splitlines()[2] == "Total distance traveled = 160.000000"
    rec = json.loads(_run([os.path.join(BIN, "riemann"), "--device", "cpu", "--integrand",
                           "table", "--profile", tri_csv, "--rule", "mid", "--n", "8e5",
                           "--json"]).splitlines()[-1])
    assert rec["analytic"] == 160.0 and rec["abs_err"] < 1e-10
    p = subprocess.run([os.path.join(BIN, "trainscan"), "--device", "cpu", "--profile", tri_csv,
                        "--parity"], capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "built-in profile" in p.stderr
