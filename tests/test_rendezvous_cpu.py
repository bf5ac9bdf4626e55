"""The native TCP rendezvous that hands the RCCL unique id to every rank of a multi-process
CLI launch (torchrun --no-python build/bin/riemann ...; csrc/runtime/comm.cpp). Replaces the
reference's MPI_Init bootstrap (riemann.cpp:62-64, 4main.c:69-71). CPU only: the unique id
comes from RCCL's bootstrap, which needs no GPU."""
from __future__ import annotations

import threading

import pytest


def _port() -> int:
    from bench import rendezvous_port  # below the ephemeral range (no self-connect)

    return rendezvous_port()


def test_rendezvous_every_rank_gets_rank0_id(native):
    world, port = 4, _port()
    got: dict[int, bytes] = {}
    errs: list[BaseException] = []

    def rank(r: int) -> None:
        try:
            got[r] = native.rendezvous_unique_id("127.0.0.1", port, r, world, 30.0)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=rank, args=(r,)) for r in (3, 1, 0, 2)]  # rank 0 not first
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not errs, errs
    assert len(got) == world
    ids = set(got.values())
    assert len(ids) == 1 and len(ids.pop()) == 128


def test_rendezvous_single_rank_needs_no_network(native):
    assert len(native.rendezvous_unique_id("127.0.0.1", _port(), 0, 1)) == 128


def test_rendezvous_times_out_without_rank0(native):
    with pytest.raises(Exception, match="timed out"):
        native.rendezvous_unique_id("127.0.0.1", _port(), 1, 2, 0.3)


def test_rendezvous_rank0_times_out_without_peers(native):
    with pytest.raises(Exception, match="timed out"):
        native.rendezvous_unique_id("127.0.0.1", _port(), 0, 3, 0.3)


def test_rendezvous_port_below_ephemeral_range():
    """Launcher ports sit below the ephemeral range with the CLIs' +17 / +19 free too: a port
    inside it can be handed to a rank's retrying connect() as its local port (self-connect;
    csrc/include/miint/net.hpp)."""
    import socket

    from bench import rendezvous_port

    with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
        low = int(f.read().split()[0])
    for _ in range(8):
        p = rendezvous_port()
        assert p + 19 < low
        for o in (0, 17, 19):
            with socket.socket() as s:
                s.bind(("", p + o))
