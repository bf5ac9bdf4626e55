"""miintrun: the `mpirun -np P` of this framework (csrc/cli/miintrun.cpp), on the CPU.

The reference is launched with Intel MPI's mpirun (riemann.cpp:62-64, 4main.c:69-71); there
is no MPI here. miintrun starts P ranks with the torchrun-style environment every entry point
reads, ends the job at the first failing rank and forwards signals. It links no HIP."""
from __future__ import annotations

import json
import os
import signal
import subprocess
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(REPO, "build", "bin", "miintrun")
RIEMANN = os.path.join(REPO, "build", "bin", "riemann")


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(RUN):
        subprocess.run(["make", "-C", REPO, "build/bin/miintrun"], check=True,
                       capture_output=True)


def test_ranks_get_the_environment():
    p = subprocess.run([RUN, "-np", "3", "sh", "-c",
                        "echo $RANK $LOCAL_RANK $WORLD_SIZE $LOCAL_WORLD_SIZE $MASTER_ADDR "
                        "$MASTER_PORT"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    rows = sorted(l.split() for l in p.stdout.splitlines())
    assert [r[:4] for r in rows] == [[str(r), str(r), "3", "3"] for r in range(3)]
    assert {r[4] for r in rows} == {"127.0.0.1"} and len({r[5] for r in rows}) == 1


def test_no_hip_linked():
    out = subprocess.run(["ldd", RUN], capture_output=True, text=True).stdout
    assert "amdhip" not in out and "rccl" not in out


def test_first_failure_ends_the_job():
    t = time.time()
    p = subprocess.run([RUN, "-np", "4", "--grace", "5", "sh", "-c",
                        'if [ "$RANK" = 2 ]; then exit 7; fi; sleep 60'],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 7 and "exited with 7" in p.stderr
    assert time.time() - t < 20  # the sleeping ranks were stopped, not waited for


def test_agreed_failure_lets_rank0_finish():
    """A rank that EXITS non-zero gives the others --linger seconds: rank 0, failing the same
    way a moment later (an agreed failure), still prints its record; a rank that never ends
    is stopped once the linger is over."""
    p = subprocess.run([RUN, "-np", "2", "--linger", "3", "sh", "-c",
                        'if [ "$RANK" = 0 ]; then sleep 0.5; echo record; fi; exit 3'],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and "record" in p.stdout
    # with 3+ ranks, the 2nd and 3rd agreed exits during the linger must not stop
    # the ranks still finishing — rank 0 exits last and its record is still printed
    p = subprocess.run([RUN, "-np", "4", "--linger", "3", "sh", "-c",
                        'if [ "$RANK" = 0 ]; then sleep 1; echo record; fi; '
                        'if [ "$RANK" = 2 ]; then sleep 0.3; fi; exit 3'],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and "record" in p.stdout, p.stderr
    t = time.time()
    p = subprocess.run([RUN, "-np", "2", "--linger", "1", "--grace", "5", "sh", "-c",
                        'if [ "$RANK" = 1 ]; then exit 3; fi; sleep 60'],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and time.time() - t < 20


def test_signals_are_forwarded():
    proc = subprocess.Popen([RUN, "-np", "2", "sleep", "60"])
    time.sleep(0.5)
    proc.send_signal(signal.SIGTERM)
    assert proc.wait(timeout=30) == 128 + signal.SIGTERM


def test_usage_and_missing_program():
    assert subprocess.run([RUN, "echo"], capture_output=True).returncode == 2
    p = subprocess.run([RUN, "-np", "2", "/nonexistent/prog"], capture_output=True, text=True,
                       timeout=30)
    assert p.returncode == 127 and "cannot run" in p.stderr


def test_host_ranks_riemann_matches_one_process():
    """`miintrun -np 3 riemann --device cpu` is `mpirun -np 3 ./riemann` with every rank
    working: rank 0 prints the one-process value (rank-order host all-reduce)."""
    if not os.path.exists(RIEMANN):
        pytest.skip("CLIs not built")
    args = [RIEMANN, "--device", "cpu", "--integrand", "pi4", "--n", "3e7", "--rule", "mid",
            "--json"]
    multi = subprocess.run([RUN, "-np", "3", *args], capture_output=True, text=True, timeout=120)
    one = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert multi.returncode == 0 and one.returncode == 0, multi.stderr + one.stderr
    m, o = json.loads(multi.stdout.splitlines()[-1]), json.loads(one.stdout.splitlines()[-1])
    assert m["ranks"] == 3 and o["ranks"] == 1
    assert m["result"] == pytest.approx(o["result"], rel=1e-15)
    assert multi.stdout.count("steps is") == 1  # rank 0 only
