"""GPU tests of the native runtime: plans, hipGraph replay, train scan, CLI tools."""
from __future__ import annotations

import json
import math
import os
import subprocess

import pytest
import torch

from cuda_v_mpi_amd import Integrator
from cuda_v_mpi_amd.utils import output

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")


def test_integrator_pi4(cuda):
    r = Integrator("pi4", n=10**9, rule="left").run()
    assert abs(r.abs_err - 1e-9) < 1e-13
    assert r.seconds_device > 0


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("fused", [False, True])
def test_plan_steps_graph_and_plain_agree(cuda, graphs, fused):
    it = Integrator("sin", n=10**8, fused=fused)
    one = it.run().value
    t = it.run_steps(9, pipeline=False, graphs=graphs)
    assert t["steps"] == 9 and t["device_ms"] > 0
    assert it.plan.host_result(it.plan.host_index_of(8, graphs)) == one


@pytest.mark.parametrize("name", ["pi4", "pi4_fp32", "sin", "table", "poly", "train"])
@pytest.mark.parametrize("collective", [False, True])
def test_chained_batches_equal_fused_bitwise(cuda, name, collective):
    """Graph batches of chained kernels (kernel k finalizes step k-1, a finalize closes the
    batch; no ticket) give every step exactly the fused kernel's value: 21 steps in batches
    of 8 (two replays of the 8-step graph + one of a 5-step graph), on one GPU and through
    the bucketed 1-rank RCCL stage."""
    dtype = "fp32" if name.endswith("_fp32") else "fp64"
    name = name.split("_")[0]
    kw = dict(n=100_000_017, rule="mid", slots=8, force_collective=collective, dtype=dtype)
    want = Integrator(name, n=100_000_017, rule="mid", dtype=dtype).run().value
    for chain in (True, False):
        it = Integrator(name, chain=chain, **kw)
        assert it.plan.chained == chain
        it.run_steps(21, pipeline=True, graphs=True)
        assert it.plan.graphs_ready, it.plan.graph_error
        assert it.plan.graph_launches == 3 and it.plan.direct_steps == 0
        for k in range(13, 21):
            assert it.plan.host_result(it.plan.host_index_of(k, True)) == want, (chain, k)


@pytest.mark.parametrize("name", ["pi4", "pi4_fp32", "pi4_fp32acc", "sin", "poly", "train",
                                  "sin_ieee", "pi4_fp32_ieee", "pi4_exact", "table",
                                  "table_fp32", "table_ieee"])
def test_multistep_batches_equal_chained_bitwise(cuda, name):
    """A graph batch as ONE persistent multi-step launch + a closing kernel (workgroups rotate
    over virtual blocks from step to step) gives every step the chained batch's value, bit for
    bit: 47 steps = two 20-step replays + a 7-step one, and 1-step batches."""
    parts = name.split("_")
    dtype = parts[1] if len(parts) > 1 and parts[1].startswith("fp") else "fp64"
    div = {"ieee": "ieee", "exact": "series_exact"}.get(parts[-1], "series")
    kw = dict(n=120_000_011, rule="mid", dtype=dtype, div=div)
    ms = Integrator(parts[0], slots=20, close="kernel", **kw)
    ch = Integrator(parts[0], slots=20, multistep=False, grid=ms.plan.grid, **kw)
    assert ms.plan.multistep and not ch.plan.multistep and ms.plan.grid == ch.plan.grid
    assert ms.plan.step_streams(20) == 1
    for it in (ms, ch):
        it.run_steps(47, pipeline=True, graphs=True)
        assert it.plan.graphs_ready, it.plan.graph_error
    assert ms.plan.graph_nodes == 2  # the persistent kernel and the closing kernel
    got = [ms.plan.host_result(ms.plan.host_index_of(k, True)) for k in range(40, 47)]
    want = [ch.plan.host_result(ch.plan.host_index_of(k, True)) for k in range(40, 47)]
    assert got == want and len(set(got)) == 1
    one = Integrator(parts[0], slots=1, **kw)
    one.run_steps(3, pipeline=True, graphs=True)
    assert one.plan.host_result(one.plan.host_index_of(2, True)) == want[0]


@pytest.mark.parametrize("shape", ["g1", "s2", "s4", "s8", "grid5", "grid17_b64",
                                   "grid100_b1024", "s8_slots64"])
@pytest.mark.parametrize("graphs", [False, True])
def test_multistep_close_in_launch_bitwise(cuda, shape, graphs):
    """close="launch" (the persistent launch's last arrivals close its batch: sc1 partials,
    sharded arrival counters, closers polling every shard) gives every step the closing
    kernel's value bit for bit: N = 1e9 and rank 0's 1/2, 1/4 and 1/8 slices, odd grids and
    64- / 1024-thread workgroups, batches of 20 (and of 64: more steps than shards, so one
    closer closes several), remainders, repeated launches (the counters re-arm)."""
    kw = dict(n=10**9, rule="left")
    name = "pi4"
    slots, steps = (64, 131) if shape.endswith("slots64") else (20, 47)
    if shape.startswith("s"):
        kw["slice_of"] = (0, int(shape[1]))
    elif shape.startswith("grid"):  # sin's 192-sample tiles: a few tiles per lane
        g = shape[4:].split("_")[0]
        name = "sin"
        kw.update(n=192 * 1000 + 77, grid=int(g), rule="mid",
                  block=int(shape.split("_b")[1]) if "_b" in shape else 256)
    a = Integrator(name, slots=slots, close="launch", **kw)
    b = Integrator(name, slots=slots, close="kernel", grid=a.plan.grid,
                   **{k: v for k, v in kw.items() if k != "grid"})
    assert a.plan.multistep and a.plan.close_in_launch and not b.plan.close_in_launch
    assert a.plan.grid == b.plan.grid
    for it in (a, b):
        it.run_steps(steps, pipeline=False, graphs=graphs)
        it.run_steps(steps, pipeline=False, graphs=graphs)
    if graphs:
        assert a.plan.graph_nodes == 1 and b.plan.graph_nodes == 2
    got = [a.plan.host_result(a.plan.host_index_of(k, graphs)) for k in range(steps)]
    want = [b.plan.host_result(b.plan.host_index_of(k, graphs)) for k in range(steps)]
    assert got == want and len(set(got)) == 1 and math.isfinite(got[0])


@pytest.mark.parametrize("name,dtype,div", [("table", "fp64", "series"),
                                            ("pi4", "fp32", "ieee")])
def test_close_in_launch_falls_back_where_it_would_spill(cuda, name, dtype, div):
    """Kernels under the 8-wave hint (the table's tiles, the fp32 IEEE tiles) would spill
    with the in-launch close: their plans keep the closing kernel, same multi-step batches."""
    a = Integrator(name, n=120_000_011, dtype=dtype, div=div, slots=20, close="launch")
    b = Integrator(name, n=120_000_011, dtype=dtype, div=div, slots=20, close="kernel")
    assert a.plan.multistep and not a.plan.close_in_launch and a.plan.grid == b.plan.grid
    for it in (a, b):
        it.run_steps(20, pipeline=False, graphs=False)
    assert a.plan.host_result(19) == b.plan.host_result(19)


@pytest.mark.parametrize("to_host", [False, True])
@pytest.mark.parametrize("close", ["kernel", "launch"])
def test_bucketed_allreduce_to_host_bitwise(cuda, to_host, close):
    """The 1-rank RCCL stage of bucketed multi-step batches: all-reduced straight into the
    pinned host slots (allreduce_to_host) or in place + a copy, closed by a kernel or in the
    launch — the same values as the single-GPU plan, bit for bit."""
    kw = dict(n=10**9 // 8, rule="left", slots=20)
    ref = Integrator("pi4", close="kernel", **kw)
    ref.run_steps(20, pipeline=False, graphs=False)
    want = ref.plan.host_result(ref.plan.host_index_of(19, False))
    it = Integrator("pi4", force_collective=True, close=close, allreduce_to_host=to_host, **kw)
    assert it.plan.bucketed and it.plan.allreduce_to_host == to_host
    assert it.plan.grid == ref.plan.grid
    for graphs in (False, True):
        it.run_steps(43, pipeline=True, graphs=graphs)
        vals = {it.plan.host_result(it.plan.host_index_of(k, graphs)) for k in range(43 - 3, 43)}
        assert vals == {want}, (graphs, vals, want)


def test_diagnose_batch_accounts_for_the_timed_batch(cuda):
    """VERDICT r5 Next #2: the diagnostic batch (events between the persistent launch, the
    close, the all-reduce and the copy) accounts for a timed batch of the same shape —
    compute + tail within 5 % of the host-timed batch — and gives its values bit for bit."""
    import statistics

    it = Integrator("pi4", n=10**9, slots=20, force_collective=True, slice_of=(0, 2))
    for _ in range(40):
        it.plan.run_steps(20, True, False)
    walls = [it.plan.run_steps(20, True, False)["wall_s"] * 1e6 for _ in range(9)]
    want = it.plan.host_result(it.plan.host_index_of(19, False))
    d = it.plan.diagnose_batch(20)
    assert d["steps"] == 20 and d["compute_us"] > 0 and d["marker_us"] >= 0
    assert d["tail_us"] == pytest.approx(d["close_us"] + d["allreduce_us"] + d["copy_us"])
    # the two passes are separate runs of the batch: they agree to their run-to-run spread,
    # with the kernel boundaries the events stood in for (a few us) as the remainder
    assert d["compute_us"] + d["tail_us"] + d["boundary_us"] == pytest.approx(d["device_us"])
    assert abs(d["boundary_us"]) < 0.03 * d["device_us"], d
    assert d["device_us"] == pytest.approx(statistics.median(walls), rel=0.05), (d, walls)
    assert d["close_us"] > 0 and d["staged_us"] >= 0.97 * d["device_us"]
    got = {it.plan.host_result(it.plan.host_index_of(k, False)) for k in range(20)}
    assert got == {want}


def test_allreduce_to_host_check_falls_back(cuda, monkeypatch):
    """A transport that cannot all-reduce into pinned memory (MIINT_FAULT_AR_HOST on rank 0:
    the plan's one-time check fails) costs a copy, not the run: the plan turns
    allreduce_to_host off before its first batch and gives the same values. (A subprocess: the
    fault variables are read once per process.)"""
    code = (
        "from cuda_v_mpi_amd import Integrator\n"
        "kw = dict(n=10**9 // 8, slots=20, force_collective=True)\n"
        "a = Integrator('pi4', **kw)\n"
        "assert a.plan.allreduce_to_host\n"
        "a.run_steps(20, pipeline=False, graphs=False)\n"
        "assert not a.plan.allreduce_to_host\n"
        "b = Integrator('pi4', n=10**9 // 8, slots=20)\n"
        "b.run_steps(20, pipeline=False, graphs=False)\n"
        "assert a.plan.host_result(19) == b.plan.host_result(19)\n"
        "print('ok')\n")
    env = dict(os.environ, MIINT_FAULT_RANK="0", MIINT_FAULT_AR_HOST="1")
    p = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=240,
                       env=env, cwd=REPO)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-2000:]


@pytest.mark.parametrize("block", [64, 256, 1024])
def test_multistep_tile_split_vs_torch(cuda, block):
    """Multi-step batches (the tile split formed once per batch, every step rotating its
    virtual blocks) at 64-, 256- and 1024-thread workgroups and a small grid: sin's
    192-sample series tiles against the fp64 torch sum of the same samples."""
    import math

    import torch

    n = 192 * 1000 + 77
    it = Integrator("sin", n=n, rule="mid", block=block, grid=5, slots=8)
    assert it.plan.multistep
    it.run_steps(8, pipeline=True, graphs=True)
    got = it.plan.host_result(it.plan.host_index_of(7, True))
    h = math.pi / n
    x = (torch.arange(n, dtype=torch.float64) + 0.5) * h
    want = math.fsum(torch.sin(x).tolist()) * h
    assert got == pytest.approx(want, rel=1e-12)


@pytest.mark.parametrize("name,div", [("pi4", "ieee")])
def test_multistep_not_where_it_does_not_pay(cuda, name, div):
    """The fp64 per-sample IEEE division measured slower as multi-step batches: its plans
    keep chained batches (multistep_pays). (The table's segment tiles joined the multi-step
    path in round 6 under the 8-wave hint: test_multistep_batches_equal_chained_bitwise.)"""
    it = Integrator(name, n=10**8, div=div)
    assert it.plan.chained and not it.plan.multistep


def test_multistep_residency_rules_the_grid(cuda):
    """The auto grid is capped at the multi-step kernel's residency (every workgroup of a
    persistent launch resident at once); an explicit grid above it runs chained batches."""
    it = Integrator("pi4", n=10**9)
    g = it.plan.grid
    assert it.plan.multistep and 0 < g <= 8 * 256 and g % 256 == 0
    big = Integrator("pi4", n=10**9, grid=g + 256)
    assert big.plan.grid == g + 256 and not big.plan.multistep and big.plan.chained
    small = Integrator("pi4", n=10**7)  # small N keeps its small auto grid
    assert small.plan.multistep and small.plan.grid <= g


@pytest.mark.parametrize("bucket", [True, False])
@pytest.mark.parametrize("graphs", [False, True])
def test_plan_rccl_stage_on_one_gpu(cuda, graphs, bucket):
    """The multi-GPU step run with a 1-rank communicator: bucketed (a batch of kernels, then
    ONE RCCL all-reduce of all their results + one copy to pinned) or per step (kernel ->
    all-reduce on the comm stream -> copy, fork/join-captured in a graph). 37 steps = two
    full batches of 16 and a partial one."""
    base = Integrator("pi4", n=10**8, rule="mid")
    want = base.run().value
    it = Integrator("pi4", n=10**8, rule="mid", force_collective=True, bucket=bucket)
    assert it.plan.collective and not it.plan.direct and it.plan.bucketed == bucket
    t = it.run_steps(37, pipeline=True, graphs=graphs)
    assert t["steps"] == 37
    if graphs:
        assert it.plan.graphs_ready, it.plan.graph_error
    for k in range(37 - it.plan.slots, 37):
        assert it.plan.host_result(it.plan.host_index_of(k, graphs)) == want


def test_watchdog_times_out_on_a_busy_stream(native, cuda):
    """The collective watchdog (wait_with_timeout: stream query, RCCL async-error check,
    abort on timeout) raises when a stream is still busy after the timeout, and returns the
    wait time once it drains. N = 2e10 keeps the stream busy for ~1.5 ms."""
    import torch

    from cuda_v_mpi_amd.models import integrands
    from cuda_v_mpi_amd.ops import kernels

    s = torch.cuda.current_stream().cuda_stream
    kernels.riemann(integrands.pi4(), 2 * 10**10)
    with pytest.raises(Exception, match="did not drain"):
        native.wait_with_timeout(s, 1e-4)
    kernels.riemann(integrands.pi4(), 10**6)
    assert native.wait_with_timeout(s, 30.0) >= 0.0
    torch.cuda.synchronize()


def native_serial_pi4_left(n):
    from cuda_v_mpi_amd import native
    m = native()
    return m.oracle.riemann_serial(m.Integrand.pi4, 0.0, 1.0, n, m.Rule.left)


def test_plan_effective_div_fallback(cuda):
    # h = 1e-3 is too coarse for the series reciprocal -> IEEE division is used
    it = Integrator("pi4", n=1000, div="series")
    assert "ieee" in str(it.plan.effective_div)
    want = native_serial_pi4_left(1000)
    assert it.run().value == pytest.approx(want, rel=1e-14)


@pytest.mark.parametrize("grid", [4096, 1000])
@pytest.mark.parametrize("chain", [True, False])
def test_table2d_plan_graph_replay(native, cuda, grid, chain):
    """Table2DPlan: one integration matches the separable oracle; timing by hipGraph replays
    of 32 integrations (chained launches + one finalize, or 32 fused launches) and by direct
    enqueue both work; the replays' last value is bitwise the direct run's."""
    plan = native.Table2DPlan(grid, 1800.0, 0, None, True, chain)
    assert plan.chained == chain
    want = native.table2d_oracle(grid)
    v = plan.run()
    assert v == pytest.approx(want, rel=1e-14)
    assert plan.time(64, True) > 0
    assert plan.last_result() == v
    assert plan.time(8, False) > 0
    assert plan.last_result() == v
    assert plan.run() == v


@pytest.mark.parametrize("grid,rows", [(4096, None), (4096, (1536, 2048)), (8192, (0, 1024)),
                                       (1000, None), (333, (10, 200))])
def test_table2d_chained_bitwise_equals_fused(native, cuda, grid, rows):
    """Raw chained launches: 3 integrations through the double buffer (launch j's workgroup 0
    closes launch j-1, a finalize closes the last) give bitwise the fused launch's value, on
    both kernels (row stream: 4096/8192 grids; tile: 1000, 333) and on row slices."""
    from cuda_v_mpi_amd.ops import kernels
    from cuda_v_mpi_amd.utils import fixtures

    v = torch.as_tensor(fixtures.profile_table(), device="cuda")
    T = kernels.outer_product(v)
    n = T.shape[0]
    r0, r1 = rows or (0, grid)
    args = (T.data_ptr(), n, n, 1800.0, 1800.0, grid, grid, r0, r1)
    nb = native.table2d_grid(n, n, 1800.0, 1800.0, grid, grid, r0, r1)
    s = torch.cuda.current_stream().cuda_stream
    slots = torch.empty(nb, dtype=torch.float64, device="cuda")
    native.fill_unset_slots(slots.data_ptr(), nb, s)
    ticket = torch.zeros(native.TICKET_WORDS, dtype=torch.int32, device="cuda")
    fused = torch.zeros(1, dtype=torch.float64, device="cuda")
    native.launch_table2d_fused(*args, slots.data_ptr(), ticket.data_ptr(), fused.data_ptr(), s)
    buf = torch.full((2, nb), float("nan"), dtype=torch.float64, device="cuda")
    out = torch.full((3,), float("nan"), dtype=torch.float64, device="cuda")
    for j in range(3):
        prev = buf[(j - 1) & 1].data_ptr() if j else 0
        native.launch_table2d_chained(*args, buf[j & 1].data_ptr(), prev,
                                      out[j - 1].data_ptr() if j else 0, s)
    native.launch_table2d_finalize(buf[0].data_ptr(), nb, out[2].data_ptr(), s)
    torch.cuda.synchronize()
    f = float(fused.item())
    assert all(float(x) == f for x in out.cpu()), (out, f)
    if rows is None and grid >= 1000:
        assert f == pytest.approx(native.table2d_oracle(grid), rel=1e-14)


def test_trainscan_native(native, cuda):
    ts = native.TrainScan(native.TrainScanConfig(), 0)
    r = ts.run()
    assert r["timeout"] == 0
    # exact knot-sampled value; the reference's sequential sum drifts to ...004030
    assert abs(r["distance"] - 122000.004) < 1e-6
    assert r["sum_of_sums"] / 1e8 == pytest.approx(109861003.621919, rel=1e-9)


def test_trainscan_beyond_2e32_samples(native, cuda):
    """3e6 samples/s: 5.4e9 samples (> 2^32), 86 GB of vel + pos on one GPU. 64-bit sample
    indices end to end; the distance is unchanged and the sum of sums scales with sps^2."""
    cfg = native.TrainScanConfig()
    cfg.steps_per_sec = 3_000_000
    r = native.TrainScan(cfg, 0).run()
    assert r["timeout"] == 0
    assert abs(r["distance"] - 122000.004) < 1e-6
    want = 109861003.621919e8 * (3_000_000 / 10_000) ** 2
    assert r["sum_of_sums"] == pytest.approx(want, rel=1e-9)


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=e)


@pytest.fixture(scope="module")
def cli_built(native):
    if not os.path.exists(os.path.join(BIN, "riemann")):
        subprocess.run(["make", "-C", REPO, "-j8", "cli"], check=True)
    return BIN


def test_cli_riemann_format(cli_built):
    p = _run([os.path.join(cli_built, "riemann")])
    assert p.returncode == 0, p.stderr
    lines = p.stdout.strip().splitlines()
    assert lines[0].endswith(" seconds")
    float(lines[0].split()[0])
    assert lines[1].startswith("The integral of f(x) from 0.0 to 3.14159265358979 with "
                               "1000000000 steps is ")
    assert float(lines[1].rsplit(" ", 1)[1]) == pytest.approx(2.0, abs=1e-11)


def test_cli_riemann_default_is_one_run(cli_built, tmp_path):
    """VERDICT r4 Next #5: the default program is the reference's single run (riemann.cpp:
    49-51,90-96): one cold + one timed integration, then exactly the two §2.6 lines — the
    one-integration-per-call harness (~450 extra integrations) runs only with --json or
    --one-shot. The --jsonl side record shows it did not run."""
    rec = tmp_path / "r.jsonl"
    p = _run([os.path.join(cli_built, "riemann"), "--jsonl", str(rec)])
    assert p.returncode == 0, p.stderr
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 2 and lines[0].endswith(" seconds")
    assert lines[1].startswith("The integral of f(x) from 0.0 to 3.14159265358979 with ")
    js = json.loads(rec.read_text().strip().splitlines()[-1])
    assert js["one_shot"] is False and "ms_one_shot" not in js
    # the whole program (process start to print) is far below what the harness would add
    # (~450 integrations of 1e9 samples ~ 35 ms of GPU time alone)
    assert js["seconds_wall"] > 0
    q = _run([os.path.join(cli_built, "riemann"), "--one-shot", "--jsonl", str(rec)])
    assert q.returncode == 0, q.stderr
    js = json.loads(rec.read_text().strip().splitlines()[-1])
    assert js["one_shot"] is True and 0 < js["ms_one_shot"] < 5.0


def test_cli_riemann_parity_single_rank_is_zero(cli_built):
    p = _run([os.path.join(cli_built, "riemann"), "--parity", "--n", "1e6"])
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip().splitlines()[1].endswith(" steps is 0")


def test_cli_cintegrate(cli_built):
    p = _run([os.path.join(cli_built, "cintegrate")])
    assert p.returncode == 0, p.stderr
    l = p.stdout.strip().splitlines()
    assert l[1] == output.fmt_cintegrate_distance(122000.004000)
    q = _run([os.path.join(cli_built, "cintegrate"), "--parity"])
    assert q.stdout.strip().splitlines()[1] == "final distance is:121999.800663"
    m = _run([os.path.join(cli_built, "cintegrate"), "--materialize"])
    assert m.stdout.strip().splitlines()[1] == "final distance is:122000.004000"


def test_cli_trainscan(cli_built):
    p = _run([os.path.join(cli_built, "trainscan"), "--json"])
    assert p.returncode == 0, p.stderr
    l = p.stdout.strip().splitlines()
    assert l[0] == "Step size of 10000"
    assert l[1].endswith(" seconds")
    assert l[2] == "Total distance traveled = 122000.004000"
    js = json.loads(l[3])
    assert js["timeout"] == 0


def test_cli_table2d_slices_sum_to_whole(cli_built):
    """miint table2d --slice R/W integrates one rank's rows of a W-GPU split on this GPU;
    the partials of all ranks add up to the whole field. 2048^2 runs 64-sample tiles from
    global memory (a 64-sample tile spans 56 cells, too many for the 32 x 32 LDS footprint),
    the 8192^2 halves 128-sample tiles staged in LDS."""
    exe = os.path.join(cli_built, "miint")
    for g, w in ((2048, 3), (8192, 2)):
        whole = _run([exe, "table2d", "--grid", str(g), "--iters", "2"])
        assert whole.returncode == 0, whole.stderr
        want = json.loads(whole.stdout.strip().splitlines()[-1])["result"]
        parts = []
        for r in range(w):
            q = _run([exe, "table2d", "--grid", str(g), "--slice", f"{r}/{w}", "--iters", "2"])
            assert q.returncode == 0, q.stderr
            parts.append(json.loads(q.stdout.strip().splitlines()[-1])["partial"])
        assert math.fsum(parts) == pytest.approx(want, rel=1e-13)


def test_cli_jsonl_appends_run_records(cli_built, tmp_path):
    """--jsonl FILE appends one record per run (SURVEY §5 metrics row), across tools; stdout
    keeps only the reference's lines unless --json is also given."""
    log = tmp_path / "runs.jsonl"
    for args in (["riemann", "--integrand", "pi4", "--n", "1e6"],
                 ["riemann", "--integrand", "pi4", "--n", "1e6", "--rule", "mid"],
                 ["cintegrate"], ["trainscan"]):
        p = _run([os.path.join(cli_built, args[0]), *args[1:], "--jsonl", str(log)])
        assert p.returncode == 0, p.stderr
        assert not any(l.startswith("{") for l in p.stdout.splitlines())
    rows = [json.loads(l) for l in log.read_text().splitlines()]
    assert [r["program"] for r in rows] == ["riemann", "riemann", "cintegrate", "trainscan"]
    want = {"n", "integrand", "dtype", "rule", "gpus", "seconds_wall", "seconds_device",
            "subintervals_per_s", "result", "abs_err", "rel_err"}
    assert want <= set(rows[0])
    assert rows[0]["abs_err"] == pytest.approx(1e-6, rel=1e-6)  # left rule: |err| = h
    assert rows[1]["rule"] == "mid" and rows[1]["abs_err"] < 1e-12
    assert rows[2]["result"] == pytest.approx(122000.004, abs=1e-6)
    assert rows[3]["distance"] == pytest.approx(122000.004, abs=1e-6)


def test_python_cli_table2d_hip(cli_built):
    p = _run(["python", "-m", "cuda_v_mpi_amd", "table2d", "--grid", "4096", "--iters", "32"],
             env={"PYTHONPATH": REPO})
    assert p.returncode == 0, p.stderr
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["backend"] == "hip" and js["rel_err_vs_oracle"] < 1e-13
    assert js["ms_per_integration"] > 0


def test_bench_two_ranks_share_one_gpu_over_gloo():
    """bench.py in the driver's launch shape (torch.distributed.run, 2 processes) on one
    GPU: torch.distributed over gloo, kernels on each rank's torch stream and one
    all_reduce per step (TorchStepper). Checks rank slicing, MAX-over-ranks timing and the
    rank-0-only JSON line; not speed (two processes time-share the card)."""
    import sys

    from bench import rendezvous_port

    port = rendezvous_port()
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr", "127.0.0.1", f"--master-port={port}",
              os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--comm",
              "torch", "--steps", "24", "--warmup", "4", "--settle-ms", "0"],
             env={"PYTHONPATH": REPO})
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 1
    js = rows[0]
    assert js["verified"] and js["n_gpus"] == 2 and js["config"]["comm"] == "torch"
    # the metric's N = 1e9 in total, split over the two ranks (strong)
    assert js["config"]["N"] == 10**9 and js["config"]["n_per_gpu"] == 5 * 10**8


def test_cli_comm_sweep(cli_built):
    """miint comm: one-rank RCCL sweep of the three collectives; every size reports a
    positive time, and the broadcast of 1 MB moves at a finite rate."""
    p = _run([os.path.join(cli_built, "miint"), "comm", "--max-bytes", "1e6", "--iters", "3"])
    assert p.returncode == 0, p.stdout + p.stderr
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]  # RCCL banner
    assert {r["op"] for r in rows} == {"allreduce", "allgather", "broadcast"}
    assert {r["bytes"] for r in rows} == {8, 64, 512, 4096, 32768, 262144, 1e6}
    for r in rows:
        assert r["gpus"] == 1 and r["us"] > 0 and math.isfinite(r["algbw_GBps"])


def test_cli_bench_close_knob(cli_built):
    """miint bench --close launch runs the in-launch close (the record says so) and gives the
    closing kernel's value bit for bit; an unknown --close is refused."""
    exe = os.path.join(cli_built, "miint")
    rows = {}
    for close in ("kernel", "launch"):
        p = _run([exe, "bench", "--integrand", "pi4", "--iters", "20", "--settle", "3",
                  "--slots", "20", "--close", close])
        assert p.returncode == 0, p.stdout + p.stderr
        rows[close] = json.loads(p.stdout.strip().splitlines()[-1])
    assert rows["kernel"]["multistep"] and rows["launch"]["multistep"]
    assert not rows["kernel"]["close_in_launch"] and rows["launch"]["close_in_launch"]
    assert rows["kernel"]["result"] == rows["launch"]["result"]
    assert rows["kernel"]["allreduce_to_host"] is False  # one GPU: no bucketed all-reduce
    bad = _run([exe, "bench", "--n", "1e6", "--iters", "2", "--close", "sometimes"])
    assert bad.returncode != 0
    # --diagnose: the diagnostic batch's stages in the record (20 steps, the slots)
    # (the default settle: ~60 ms of steps first, so both passes run at the settled clock)
    p = _run([exe, "bench", "--integrand", "pi4", "--iters", "200", "--slots", "20",
              "--diagnose"])
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["diag_steps"] == 20 and d["diag_compute_us"] > 0 and d["diag_close_us"] > 0
    assert d["diag_device_us"] == pytest.approx(d["diag_compute_us"] + d["diag_tail_us"]
                                                + d["diag_boundary_us"])
    assert abs(d["diag_boundary_us"]) < 0.03 * d["diag_device_us"], d
    # one GPU, no collective: the all-reduce stage is empty once the event's price is off
    assert d["diag_marker_us"] > 0 and d["diag_allreduce_us"] < 1.5, d
    # 20 steps of 1e9 samples: ~1.4 ms; the batch is within 20 % of the timed steps
    assert d["diag_device_us"] == pytest.approx(20 * d["ms_per_integration"] * 1e3, rel=0.2)
    assert "diag_steps" not in rows["kernel"]


def test_cli_selfcheck(cli_built):
    p = _run([os.path.join(cli_built, "miint"), "selfcheck"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "SELFCHECK OK" in p.stdout


def _torchrun(nproc, args, timeout=300):
    from bench import rendezvous_port

    port = rendezvous_port()
    return _run(["python", "-m", "torch.distributed.run", "--nnodes=1",
                 f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
                 "--master-port", str(port)] + args, timeout=timeout)


def test_bench_torchrun_single_rank(native, cuda):
    p = _torchrun(1, [os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "16",
                      "--warmup", "2"])
    assert p.returncode == 0, p.stderr[-2000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["verified"] and js["n_gpus"] == 1


def test_bench_two_ranks_shared_gpu_torch_comm(native, cuda):
    """Two processes on one GPU: rank slicing + torch.distributed (gloo) all_reduce of the
    per-rank kernel partials; --samples is the total N, halved per rank."""
    p = _torchrun(2, [os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                      "--comm", "torch", "--steps", "12", "--warmup", "2", "--samples", "2e8"])
    assert p.returncode == 0, p.stderr[-3000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["n_gpus"] == 2 and js["config"]["N"] == 200_000_000 and js["verified"]
    assert js["config"]["n_per_gpu"] == 100_000_000


def test_bench_native_comm_failure_falls_back_to_torch(native, cuda):
    """Two ranks on one GPU with the native communicator: RCCL rejects ranks that share a
    device ("invalid usage") on both ranks, the ranks agree on the failure over the gloo
    group and run the torch.distributed step path instead; the record names the fallback and
    is NOT verified (native_comm_verified false), though its headline numbers check out."""
    p = _torchrun(2, [os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                      "--comm", "native", "--steps", "12", "--warmup", "2", "--samples", "2e8",
                      "--settle-ms", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    assert js["headline_verified"] and js["n_gpus"] == 2 and js["config"]["comm"] == "torch"
    assert js["comm_fallback"] and "falling back to --comm torch" in p.stderr
    assert not js["verified"] and not js["native_comm_verified"]


@pytest.mark.parametrize("bucket", [True, False])
def test_bench_force_collective_graph(native, cuda, bucket):
    """The 1-rank RCCL stage with the multi-step batches replayed as hipGraphs
    (--graph-batches; the default launches them directly, test_bench_contract)."""
    p = _run(["python", os.path.join(REPO, "bench.py"), "--steps", "40", "--warmup", "8",
              "--force-collective", "--graph-batches"] + ([] if bucket else ["--no-bucket"]))
    assert p.returncode == 0, p.stderr[-2000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])
    bad = [k for k, v in js.items() if isinstance(v, dict) and v.get("verified") is False]
    assert "extras_error" not in js, js["extras_error"]
    assert js["verified"] and not bad, bad
    assert js["config"]["graphs"] and js["config"]["pipeline"]
    assert js["config"]["batch_launch"] == "graph"
    assert js["config"]["bucketed_allreduce"] == bucket


def test_bench_contract(native, cuda):
    p = _run(["python", os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "3"])
    assert p.returncode == 0, p.stderr
    js = json.loads(p.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in js
    assert js["n_gpus"] == 1 and js["steps"] == 20 and js["verified"]
    assert js["value"] > 1e11
    # the 20 timed steps are ONE multi-step batch (slots = 48): one persistent launch of the
    # 20 steps and its closing kernel, enqueued directly (measured faster than the same two
    # kernels as a graph replay, profiles/r5/graph_vs_direct.md)
    assert js["direct_steps_timed"] == 20 and js["graph_replays_timed"] == 0
    assert js["config"]["batch_launch"] == "direct" and js["config"]["multistep"]
    assert js["config"]["graphs"] is False
    # the settle, then the timed pattern once more on its own before the clock (untimed)
    assert js["warmup_rearm_batch"] and js["warmup_settle_steps"] >= 2 * 20
    assert js["pre_clock_barrier"] == "host"  # one GPU: no device barrier to move behind
    # the record carries what the headline rests on: IEEE-division speed and per-point ulp
    assert js["ieee_div_value"] > 1e11 and js["ieee_div"]["abs_err"] < 2e-9
    # the headline division (series_exact): per point within 3 ulp of the IEEE path's own
    # values, within 1.5 of the true value; the faster g-fold (series) rides along as an extra
    assert js["config"]["division"] == "series_exact" and js["per_point"]["division"] == "series_exact"
    assert js["per_point_max_ulp"] <= 3.0 and js["per_point_vs_true_max_ulp"] <= 1.5
    assert js["series_div"]["verified"] and js["series_div"]["per_point"]["max_ulp"] <= 5.0
    b3 = js["baseline3_strong_1e10"]
    assert b3["N"] == 10**10 and abs(b3["abs_err"] - 1e-10) < 1e-13 and b3["value"] > 1e11
    assert js["rccl_version"] and js["per_rank_ms"] and js["launcher"] == "single"


def test_compare_gpu_vs_host(native, cuda):
    """`compare` (the reference's CUDA-vs-MPI comparison, measured on one box): the GPU row,
    the host engine row and the reference program on threads all integrate sin on [0, pi] to
    the same value; the GPU is faster than the host cores."""
    p = subprocess.run(["python", "-m", "cuda_v_mpi_amd", "compare", "--n", "1e8", "--reps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    rows = [json.loads(x) for x in p.stdout.splitlines()]
    by = {r["side"]: r for r in rows if "side" in r}
    assert set(by) == {"host", "reference-program", "gpu"}
    for r in by.values():
        assert abs(r["value"] - 2.0) < 1e-12, r
    assert by["reference-program"]["value"] == native.oracle.riemann_mpi_parity(8, 1e8)
    assert rows[-1]["speedup_gpu_vs_host"] > 1.0


@pytest.mark.parametrize("block", [64, 128, 512, 1024])
def test_block_sizes(native, cuda, block):
    """--block (the reference's SP, cintegrate.cu:17-18,124-127): every supported workgroup
    size integrates correctly, the chained graph batch equals the one-launch fused form
    bitwise at that size, and unsupported sizes are refused with the list of valid ones."""
    from cuda_v_mpi_amd import Integrator

    n = 10**8 + 17
    it = Integrator("pi4", n=n, rule="mid", block=block)
    assert it.plan.block == block
    one = it.run().value
    assert one == pytest.approx(math.pi, abs=1e-13)
    it.plan.run_steps(5, False, True)  # chained graph batch
    assert it.plan.host_result(it.plan.host_index_of(4, True)) == one
    s = Integrator("sin", n=10**7 + 3, rule="mid", block=block, div="ieee").run().value
    assert s == pytest.approx(2.0, abs=1e-12)
    with pytest.raises(RuntimeError, match="64, 128, 256, 512 or 1024"):
        Integrator("pi4", n=n, block=192)


@pytest.mark.parametrize("streams", [2, 3, 4])
def test_step_streams_bitwise(native, cuda, streams):
    """Chained graph batches dealt over several streams (each its own chain, own partials,
    own finalize; the compute stream joins them) give every step exactly the one-stream
    result, bitwise — including remainder batches whose step count the streams do not
    divide. (Chained batches: multistep=False; a multi-step batch is one launch.)"""
    from cuda_v_mpi_amd import Integrator

    n = 10**8 + 7
    ref = Integrator("pi4", n=n, rule="mid", slots=48, step_streams=1, multistep=False)
    assert ref.plan.step_streams(48) == 1
    ref.plan.run_steps(48, False, True)
    want = [ref.plan.host_result(ref.plan.host_index_of(k, True)) for k in range(48)]
    assert len(set(want)) == 1
    it = Integrator("pi4", n=n, rule="mid", slots=48, step_streams=streams, multistep=False)
    assert it.plan.step_streams(48) == streams
    for steps in (48, 29, 5):
        it.plan.run_steps(steps, False, True)
        got = [it.plan.host_result(it.plan.host_index_of(k, True)) for k in range(steps)]
        assert got == want[:steps]


def test_step_streams_auto_policy(native, cuda):
    """Auto (chained batches): four streams below 6e8 samples per step, one at or above (N =
    1e9 on one GPU); a multi-step batch (the default) is one launch on one stream."""
    from cuda_v_mpi_amd import Integrator

    kw = dict(n=10**9, slots=48, multistep=False)
    assert Integrator("pi4", **kw).plan.step_streams(48) == 1
    assert Integrator("pi4", slice_of=(0, 8), **kw).plan.step_streams(48) == 4
    assert Integrator("pi4", slice_of=(0, 8), **kw).plan.step_streams(3) == 3
    assert Integrator("pi4", n=10**9, slots=48, slice_of=(0, 8)).plan.step_streams(48) == 1


def test_table2d_step_streams_equal(native, cuda):
    """The 2-D replay on 1, 2 and 4 chained streams and as one multi-step launch: the same 32
    results, bitwise."""
    res = []
    ms = native.Table2DPlan(4096, 1800.0, 0, None, True, True, 2)
    assert ms.multistep and ms.step_streams == 1
    for ss in (1, 2, 4):
        p = native.Table2DPlan(4096, 1800.0, 0, None, True, True, ss, multistep=False,
                               min_wg=ms.min_wg)
        assert p.step_streams == ss and not p.multistep
        p.time(p.graph_steps, True)
        res.append(p.last_result())
    ms.time(ms.graph_steps, True)
    res.append(ms.last_result())
    assert res[0] == res[1] == res[2] == res[3] == native.table2d_oracle(4096)


@pytest.mark.parametrize("g,sl", [(4096, (0, 8)), (4096, (7, 8)), (5000, (3, 8)), (4096, (0, 1)),
                                  (4095, (0, 4))])
def test_table2d_multistep_equals_chained(native, cuda, g, sl):
    """Row slices and grids of several shapes: the multi-step replay (every integration
    re-stages its footprint in one persistent launch) gives the chained replay's partial,
    bitwise (the chained plan given the multi-step plan's shape: a multi-step plan takes the
    most rows per wave that fit, min_wg 1)."""
    b = native.Table2DPlan(g, 1800.0, 0, None, True, True, 1, sl[0], sl[1])
    assert b.multistep and b.min_wg == 1
    a = native.Table2DPlan(g, 1800.0, 0, None, True, True, 1, sl[0], sl[1], multistep=False,
                           min_wg=b.min_wg)
    assert a.workgroups == b.workgroups
    a.time(a.graph_steps, True)
    b.time(b.graph_steps, True)
    assert a.last_result() == b.last_result()


@pytest.mark.parametrize("g,sl", [(4096, (0, 8)), (4096, (5, 8)), (4096, (1, 4)), (4095, (0, 2)),
                                  (5000, (3, 8))])
@pytest.mark.parametrize("phases", [2, 3, 4, 16, 32])
def test_table2d_multistep_phases_bitwise(native, cuda, g, sl, phases):
    """Step phases: several workgroups per row-stream block, each running every phases-th
    integration of the replay (32 integrations: 2, 3 and 4 phases, the last leaving 2 steps
    for some phases) — every integration's value bitwise the one-phase launch's, and the
    chained replay's."""
    a = native.Table2DPlan(g, 1800.0, 0, None, True, True, 1, sl[0], sl[1], multistep=False,
                           min_wg=1)
    one = native.Table2DPlan(g, 1800.0, 0, None, True, True, 1, sl[0], sl[1], phases=1)
    many = native.Table2DPlan(g, 1800.0, 0, None, True, True, 1, sl[0], sl[1], phases=phases)
    assert one.multistep and one.phases == 1 and many.phases == phases
    for p in (a, one, many):
        p.time(p.graph_steps, True)
    assert a.last_result() == one.last_result() == many.last_result()
    assert many.run() == one.run()


def test_table2d_multistep_auto_phases(native, cuda):
    """Auto: kT2AutoPhases (16) step phases on the most rows per wave that fit (16 rows on
    4096^2: 16 x 8 = 128 blocks for the 1/8 row slice, 16 x 64 for the whole field), doubled
    while the launch holds fewer than 4096 workgroups (the 1/8 slice: 32) — the fastest
    measured (profiles/r4/t2d_slice_shapes.jsonl, t2d_phases_explicit.jsonl,
    profiles/r5/t2d/n_t2d_steps.jsonl) — and the same values as one phase."""
    p = native.Table2DPlan(4096, 1800.0, 0, None, True, True, 1, 0, 8)
    assert p.multistep and p.phases == 32 and p.min_wg == 1 and p.workgroups == 128
    full = native.Table2DPlan(4096)
    assert full.multistep and full.phases == 16 and full.workgroups == 1024
    one = native.Table2DPlan(4096, phases=1)
    full.time(full.graph_steps, True)
    one.time(one.graph_steps, True)
    assert full.last_result() == one.last_result() == native.table2d_oracle(4096)
    # an explicit shape target is kept
    assert native.Table2DPlan(4096, 1800.0, 0, None, True, True, 1, 0, 8,
                              min_wg=512).workgroups == 512


def test_table2d_replay_steps_adapt_to_the_share(native, cuda):
    """A multi-step replay holds at least kReplaySamples = 2^33 samples (doubling from 32 up to
    1024 integrations): 512 for the whole 4096^2 field, 1024 for its 1/8 row slice. Chained
    replays keep 32 (one kernel node per integration); an explicit count is kept. Every
    replay size gives the same values, bitwise."""
    full = native.Table2DPlan(4096)
    s8 = native.Table2DPlan(4096, 1800.0, 0, None, True, True, 1, 0, 8)
    s8_32 = native.Table2DPlan(4096, 1800.0, 0, None, True, True, 1, 0, 8, graph_steps=32)
    chained = native.Table2DPlan(4096, multistep=False)
    assert (full.graph_steps, s8.graph_steps, s8_32.graph_steps) == (512, 1024, 32)
    assert chained.graph_steps == 32 and not chained.multistep
    for p in (full, s8, s8_32):
        p.time(p.graph_steps, True)
    assert full.last_result() == native.table2d_oracle(4096)
    assert s8.last_result() == s8_32.last_result() == s8.run()
    with pytest.raises(Exception):
        native.Table2DPlan(4096, graph_steps=1025)
    # every rank of an uneven split replays the same count (its all-reduce covers them all)
    assert {native.Table2DPlan(4095, 1800.0, 0, None, True, True, 1, r, 8).graph_steps
            for r in range(8)} == {1024}
    assert native.Table2DPlan(1000).graph_steps == 32  # the tile kernel: chained replays


def test_table2d_slice_with_forced_rccl_stage(native, cuda):
    """A row slice with a 1-rank RCCL communicator and force_collective (tools/t2d_strong.py's
    rehearsal of one rank of a G-GPU run): every replay ends in the bucketed all-reduce +
    copy, and the partial is bitwise the plain slice's."""
    from cuda_v_mpi_amd.parallel.dist import DistContext, native_comm

    comm = native_comm(DistContext())
    forced = native.Table2DPlan(4096, 1800.0, 0, comm, True, True, 0, 0, 8, force_collective=True)
    plain = native.Table2DPlan(4096, 1800.0, 0, None, True, True, 0, 0, 8)
    quiet = native.Table2DPlan(4096, 1800.0, 0, comm, True, True, 0, 0, 8)
    assert forced.collective and forced.bucketed and forced.multistep
    assert not plain.collective and not quiet.collective and not quiet.bucketed
    assert (forced.row0, forced.row1) == (plain.row0, plain.row1) == (0, 512)
    for p in (forced, plain):
        p.time(p.graph_steps, True)
    assert forced.last_result() == plain.last_result() == forced.run() == plain.run()


def test_table2d_multistep_past_residency(native, cuda):
    """8192^2 in one piece: more row-stream workgroups than the GPU holds at once. The
    multi-step replay needs no residency (no workgroup waits on another): the plan runs it,
    and every value is bitwise the chained replay's at the same shape."""
    p = native.Table2DPlan(8192, 1800.0, 0, None, True, True, 0)
    assert p.multistep and p.phases == 16 and p.step_streams == 1
    assert p.workgroups > p.resident_per_cu * native.device_info(0)["num_cus"]
    c = native.Table2DPlan(8192, 1800.0, 0, None, True, True, 1, multistep=False,
                           min_wg=p.min_wg)
    assert not c.multistep and c.workgroups == p.workgroups
    p.time(p.graph_steps, True)
    c.time(c.graph_steps, True)
    assert p.last_result() == c.last_result()
    assert abs(p.last_result() - native.table2d_oracle(8192)) <= 1e-12 * native.table2d_oracle(8192)


@pytest.mark.parametrize("graphs", [False, True])
def test_host_direct_off_copies_batch_results(native, cuda, graphs):
    """a single-GPU plan built with host_direct = false keeps its results in device
    slots; a multi-step (or chained) batch must still copy them into pinned memory."""
    m = native
    cfg = m.RiemannConfig()
    cfg.integrand, cfg.n, cfg.rule = m.Integrand.pi4, 100_000_017, m.Rule.mid
    cfg.host_direct = False
    cfg.slots = 8
    p = m.RiemannPlan(cfg, 0)
    assert not p.direct and p.multistep
    want = p.run()
    p.run_steps(11, False, graphs)
    for k in range(8, 11):
        assert p.host_result(p.host_index_of(k, graphs)) == want, k


def test_full_grid_when_batches_never_run_multistep(cuda):
    """the multi-step residency cap applies only to plans whose batches can run as
    multi-step launches; an unfused plan keeps the full auto grid."""
    capped = Integrator("pi4", n=10**9)
    full = Integrator("pi4", n=10**9, fused=False)
    assert capped.plan.multistep and not full.plan.multistep and not full.plan.chained
    assert full.plan.grid > capped.plan.grid and full.plan.grid % 256 == 0


@pytest.mark.parametrize("mode", ["direct", "direct_poll", "graph", "graph_poll"])
def test_time_one_shot(cuda, mode):
    """One integration per call, launch to pinned result (the reference's timing unit): every
    form returns the integration's value, and the host interval covers the device span."""
    it = Integrator("pi4", n=10**9, multistep=False)
    r = it.plan.time_one_shot(10, mode, 50)
    assert abs(abs(r["value"] - math.pi) - 1e-9) < 1e-13
    assert r["reps"] == 10 and 20.0 < r["median_us"] < 5000.0
    # a synchronised call's host interval covers the device span; a polled one may end before
    # the kernel (or the graph's closing kernel) has drained and the end event fired
    if not mode.endswith("_poll"):
        assert 0 < r["device_median_us"] <= r["median_us"] + 1.0
    else:
        assert 0 < r["device_median_us"] <= r["median_us"] + 20.0


def test_cli_riemann_reports_one_shot(cli_built):
    p = _run([os.path.join(cli_built, "riemann"), "--integrand", "pi4", "--json", "--iters", "20"])
    assert p.returncode == 0, p.stderr
    js = json.loads(p.stdout.strip().splitlines()[-1])
    # the one-shot is timed after 400 settling calls, the 20 steps from a cold clock (~25 ms
    # of ramp, profiles/r4/oneshot_trace.md): the same order, not the same clock
    assert js["ms_one_shot"] > js["device_ms"] * 0.6 and js["ms_one_shot"] < 5.0
    assert js["comm"] == "none" and js["rccl_world"] == 0 and js["ranks_share_gpus"] is False
