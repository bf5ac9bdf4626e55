"""Multi-rank agreement on the CPU: the reported time is the slowest rank's, RCCL's transport is
read from its INIT log, and the bench's transport check fails a node-local run over a network.

The reference's rank 0 stops its clock only after every worker's MPI_Recv (riemann.cpp:82-93),
so its "seconds" always covers the slowest worker; these tests hold the native tools to the
same (a rank made slow with MIINT_FAULT_RANK / MIINT_FAULT_DELAY_MS, miint/fault.hpp).
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
sys.path.insert(0, REPO)

import bench  # noqa: E402

# Lines as RCCL 2.2x writes them under NCCL_DEBUG=INFO, NCCL_DEBUG_SUBSYS=INIT (the socket
# ones are from profiles/r3/shared_rccl, two ranks sharing one GPU; the xGMI ones are the
# format of the P2P transport's connect line).
NET_LOG = """\
host:1:1 [0] NCCL INFO NET/Socket : Using [0]lo:127.0.0.1<0>
host:1:1 [0] NCCL INFO comm 0x5566 rank 0 nRanks 2 nNodes 2 localRanks 1 localRank 0 MNNVL 0
host:1:1 [0] NCCL INFO Channel 00/0 : 1[0] -> 0[0] [receive] via NET/Socket/0
host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0
host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[0] [send] via NET/Socket/0
host:1:1 [0] NCCL INFO comm 0x5566 rank 0 nranks 2 cudaDev 0 busId 5000 - Init COMPLETE
"""
P2P_LOG = """\
host:7:7 [0] NCCL INFO comm 0x77 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0
host:7:7 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read
host:7:7 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC/read
host:7:7 [0] NCCL INFO Channel 00/0 : 7[7] -> 0[0] via P2P/IPC/read
host:7:7 [0] NCCL INFO Channel 02/0 : 0[0] -> 2[2] via P2P/direct pointer
host:7:7 [0] NCCL INFO comm 0x77 rank 0 nranks 8 cudaDev 0 busId 1000 - Init COMPLETE
"""


def test_parse_rccl_log_net(native):
    t = native.parse_rccl_log(NET_LOG)
    assert t["transport"] == "NET/Socket" and t["uses_net"]
    assert (t["nranks"], t["nnodes"], t["local_ranks"]) == (2, 2, 1)
    assert t["connections"] == 3 and t["comms"] == 1


def test_parse_rccl_log_p2p(native):
    t = native.parse_rccl_log(P2P_LOG)
    assert t["transport"] == "P2P/IPC+P2P/direct" and not t["uses_net"]
    assert (t["nranks"], t["nnodes"], t["local_ranks"]) == (8, 1, 8)
    assert t["connections"] == 4


def test_parse_rccl_log_empty(native):
    t = native.parse_rccl_log("")
    assert t["transport"] == "" and t["nnodes"] == 0 and not t["uses_net"]


def test_transport_check(native, monkeypatch):
    net, p2p = native.parse_rccl_log(NET_LOG), native.parse_rccl_log(P2P_LOG)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    # two ranks of one node on distinct GPUs over sockets: the record cannot stand
    assert "expected P2P" in bench.transport_check(2, False, net)
    # ... unless they share a GPU (MIINT_OVERSUBSCRIBE: sockets are the transport then)
    assert bench.transport_check(2, True, net) is None
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert bench.transport_check(8, False, p2p) is None
    assert bench.transport_check(1, False, net) is None
    # fail-closed (VERDICT r4 Weak #2): distinct local GPUs with no transport evidence — no
    # RCCL log, or a log without a single peer connection — cannot count as xGMI
    assert "transport unknown" in bench.transport_check(8, False, {})
    empty = native.parse_rccl_log("")
    assert "transport unknown" in bench.transport_check(8, False, empty)
    assert "no peer connection" in bench.transport_check(8, False, dict(empty, log="/tmp/x.log"))
    # ... but ranks sharing one GPU, a 1-rank job and a gloo-only job (no RCCL) need none
    assert bench.transport_check(8, True, {}) is None
    assert bench.transport_check(1, False, {}) is None
    assert bench.transport_check(8, False, {}, rccl=False) is None
    # shared host memory between ranks on distinct GPUs (P2P disabled) is not xGMI either
    shm = native.parse_rccl_log(P2P_LOG.replace("via P2P/IPC", "via SHM/direct/direct"))
    assert shm["transport"].startswith("SHM") and not shm["uses_net"]
    assert "expected P2P" in bench.transport_check(8, False, shm)
    # a multi-node job legitimately crosses nodes over the network
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert bench.transport_check(2, False, net) is None


def test_record_verified_fails_on_comm_fallback():
    """VERDICT r5 Next #3: a run that survived a native-communicator failure on the
    torch.distributed data plane keeps its record but is not verified."""
    assert bench.record_verified(True, True, None, None)
    assert not bench.record_verified(True, True, None, "RuntimeError: ncclCommInitRank failed")
    assert not bench.record_verified(True, True, "transport is NET/Socket", None)
    assert not bench.record_verified(True, False, None, None)
    assert not bench.record_verified(False, True, None, None)


def _run(args, env):
    e = dict(os.environ, **env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    p = subprocess.run(args, capture_output=True, text=True, timeout=120, env=e)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("prog", ["riemann", "cintegrate"])
def test_slow_rank_sets_the_reported_time(prog):
    """Rank 1 of 2 holds its end-of-timing clock back by 400 ms: rank 0's record must report
    at least that (the max over ranks), and a run without the fault must not."""
    args = [os.path.join(BIN, "miintrun"), "-np", "2", "--", os.path.join(BIN, prog),
            "--device", "cpu", "--threads", "1", "--json"]
    if prog == "riemann":
        args += ["--integrand", "pi4", "--n", "1e6"]
    slow = _run(args, {"MIINT_FAULT_RANK": "1", "MIINT_FAULT_DELAY_MS": "400"})
    fast = _run(args, {})
    assert len(slow) == 1 and len(fast) == 1  # rank 0 prints
    assert slow[0]["host_ms"] >= 400.0
    assert fast[0]["host_ms"] < 400.0
    assert slow[0]["result"] == fast[0]["result"]


def test_native_transport_error_matches_bench(native):
    """The native CLIs' verdict (csrc/runtime/agree.cpp transport_error, written into every
    multi-rank record as transport_verified / transport_error) follows bench.py's rules."""
    for text, world, local, share in ((NET_LOG, 2, 2, False), (NET_LOG, 2, 2, True),
                                      (P2P_LOG, 8, 8, False), ("", 8, 8, False),
                                      ("", 8, 8, True), ("", 1, 1, False), (NET_LOG, 2, 1, False)):
        import os

        os.environ["LOCAL_WORLD_SIZE"] = str(local)
        try:
            py = bench.transport_check(world, share, native.parse_rccl_log(text))
        finally:
            del os.environ["LOCAL_WORLD_SIZE"]
        cc = native.transport_error(text, world, local, share)
        assert (py is None) == (cc == ""), (text[:40], world, local, share, py, cc)
    assert "transport unknown" in native.transport_error("", 8, 8, False)
    shm_log = P2P_LOG.replace("via P2P/IPC", "via SHM/direct/direct")
    assert "expected P2P" in native.transport_error(shm_log, 8, 8, False)
    assert native.transport_error(P2P_LOG, 8, 8, False) == ""
    assert "expected P2P" in native.transport_error(NET_LOG, 2, 2, False)


def test_replica_digest(native):
    """trainscan --replicate's per-rank fingerprint (runtime/trainscan.cpp digest_table): FNV-1a
    64 over the little-endian bytes of every double, a compensated sum, and the elements at
    0, n/4, n/2, 3n/4, n-1 — equal hashes iff bitwise-equal copies."""
    import struct

    v = [math.sin(0.001 * i) * 1e5 for i in range(10_001)]
    h = 1469598103934665603
    for x in v:
        for byte in struct.pack("<d", x):
            h = ((h ^ byte) * 1099511628211) & (2**64 - 1)
    d = native.replica_digest(v)
    assert d["hash"] == h and d["n"] == len(v)
    assert d["sum"] == math.fsum(v)
    n = len(v)
    assert d["at"] == [v[0], v[n // 4], v[n // 2], v[3 * (n // 4)], v[n - 1]]
    w = list(v)
    w[5000] = math.nextafter(w[5000], math.inf)  # one ulp anywhere changes the hash
    assert native.replica_digest(w)["hash"] != h
