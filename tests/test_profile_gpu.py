"""User velocity profiles on the MI355X: the GPU Riemann table integrand, the materialised
cintegrate path and the train scan (every algorithm) integrate a profile read from a file."""
from __future__ import annotations

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
TRIANGLE = [0.0, 10.0, 20.0, 30.0, 40.0, 30.0, 20.0, 10.0, 0.0]  # integral 160


@pytest.fixture
def tri_csv(tmp_path):
    p = tmp_path / "tri.csv"
    p.write_text("\n".join(str(v) for v in TRIANGLE) + "\n")
    return str(p)


@pytest.mark.parametrize("extra", [[], ["--materialize"]])
def test_cintegrate_profile(cuda, tri_csv, extra):
    p = subprocess.run([os.path.join(BIN, "cintegrate"), "--profile", tri_csv, *extra],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.splitlines()[1] == "final distance is:160.000000"


@pytest.mark.parametrize("algo", ["fused", "onepass", "lookback"])
def test_trainscan_profile(native, cuda, algo):
    c = native.TrainScanConfig()
    c.table = TRIANGLE
    c.seconds = 8
    c.algo = algo
    r = native.TrainScan(c, 0).run()
    assert r["distance"] == pytest.approx(160.0, rel=1e-12)
    host = native.host_trainscan(10000, 8, native.HostPool(2), None, False, TRIANGLE)
    assert r["sum_of_sums"] == pytest.approx(host["sum_of_sums"], rel=1e-11)


def test_trainscan_profile_too_short(native, cuda):
    c = native.TrainScanConfig()
    c.table = TRIANGLE  # 8 s of table, 1800 s asked for
    with pytest.raises(RuntimeError, match="exceeds the table"):
        native.TrainScan(c, 0)
