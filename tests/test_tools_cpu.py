"""CPU tests of the profiling report tools (tools/roofline.py, tools/summarize_counters.py,
tools/gap_report.py) on synthetic rocprofv3 output trees: the speed-of-light arithmetic the
committed profiles/r2/roofline.md rests on, and the timed-region gap report."""
from __future__ import annotations

import csv
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
KERNEL = "void miint::(anonymous namespace)::riemann_chained_kernel<(miint::DivMode)1, miint::Pi4>(x)"


def _write_group(d, counters, start=1000, end=1000 + 359_400):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Correlation_Id", "Kernel_Name",
                                          "Counter_Name", "Counter_Value", "Start_Timestamp",
                                          "End_Timestamp"])
        w.writeheader()
        for name, value in counters.items():
            w.writerow({"Dispatch_Id": 1, "Correlation_Id": 1, "Kernel_Name": KERNEL,
                        "Counter_Name": name, "Counter_Value": value,
                        "Start_Timestamp": start, "End_Timestamp": end})


def test_roofline_valu_bound_with_transcendentals(tmp_path):
    # the IEEE-division kernel's measured counters: 1.642e8 VALU of which 1.5625e7 v_rcp_f64,
    # 359.4 us -> bound (4 x 1.4795e8 + 16 x 1.5625e7) / (1024 x 2.4e9) = 343.5 us, 96 %
    _write_group(str(tmp_path / "pi4_ieee_G1"),
                 {"SQ_INSTS_VALU": 1.642e8, "SQ_INSTS_VALU_TRANS_F64": 1.5625e7})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline.py"),
                          str(tmp_path)], capture_output=True, text=True, check=True).stdout
    row = [ln for ln in out.splitlines() if ln.startswith("| pi4_ieee")]
    assert len(row) == 1, out
    cells = [c.strip() for c in row[0].strip("|").split("|")]
    assert cells[2] == "359.4"           # median dispatch, us
    assert cells[4] == "10.51"           # VALU per sample (N = 1e9)
    assert cells[5] == "343.5"           # VALU issue bound, us
    assert cells[8] == "96%"


def test_roofline_hbm_bound(tmp_path):
    # a 288 MB store stream in 46.9 us: HBM bound 288e6 / 8e12 = 36 us -> 77 %
    _write_group(str(tmp_path / "trainscan_G3"),
                 {"SQ_INSTS_VALU": 8.51e6, "FETCH_SIZE": 415.2, "WRITE_SIZE": 281250.0},
                 end=1000 + 46_900)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline.py"),
                          str(tmp_path)], capture_output=True, text=True, check=True).stdout
    row = [ln for ln in out.splitlines() if ln.startswith("| trainscan")][0]
    cells = [c.strip() for c in row.strip("|").split("|")]
    assert cells[7] == "36.1" and cells[8] == "77%"


def test_summarize_counters_table(tmp_path):
    _write_group(str(tmp_path / "pi4_ieee_G1"), {"SQ_INSTS_VALU": 1.642e8})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_counters.py"),
                          str(tmp_path)], capture_output=True, text=True, check=True).stdout
    assert "riemann_chained_kernel<(DivMode)1, Pi4>" in out and "SQ_INSTS_VALU=1.642e+08" in out


def _dispatches(n=4, dur=72_000, gap=500):
    """n back-to-back dispatches (ns timestamps), the last one 'gap' ns after its predecessor."""
    out, t = [], 10_000
    for i in range(n):
        if i == n - 1:
            t += gap
        out.append((KERNEL if i < n - 1 else "finalize_kernel(double const*, int)", t, t + dur))
        t += dur
    return out


def _gap_report(d, last):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gap_report.py"), str(d),
                           "--last", str(last)], capture_output=True, text=True, check=True).stdout


def test_gap_report_rocpd_database(tmp_path):
    # rocprofv3's default output: a rocpd SQLite database with a `kernels` view
    import sqlite3

    db = sqlite3.connect(str(tmp_path / "run_results.db"))
    db.execute("create table kernels (name text, start integer, end integer)")
    db.executemany("insert into kernels values (?, ?, ?)", _dispatches())
    db.commit()
    db.close()
    out = _gap_report(tmp_path, 3)
    assert out.count("riemann_chained_kernel<(DivMode)1, Pi4>") == 2, out
    assert "gaps: max 0.50 us" in out and "span 216.5 us over 3 dispatches" in out


def test_gap_report_csv_trace(tmp_path):
    with open(tmp_path / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for n, s, e in _dispatches(gap=0):
            w.writerow({"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e})
    out = _gap_report(tmp_path, 4)
    assert "gaps: max 0.00 us" in out and "over 4 dispatches" in out


def test_shared_rccl_report_flags_records_above_one_rank(tmp_path):
    """tools/shared_rccl_report.py: a multi-rank record on the shared GPU may not beat its
    tool's one-rank rate (every tool reports the slowest rank behind a barrier); the report
    marks one that does and exits 1."""
    import json

    recs = [
        {"step": "riemann_np1", "gpus": 1, "comm": "none", "subintervals_per_s": 1.2e13},
        {"step": "riemann_np2", "gpus": 2, "comm": "rccl", "rccl_world": 2,
         "rccl_transport": "NET/Socket", "rccl_nnodes": 2, "ranks_share_gpus": True,
         "subintervals_per_s": 1.1e13},
        {"step": "miint_bench_np1", "gpus": 1, "subintervals_per_s": 1.3e13},
        {"step": "miint_bench_np2", "gpus": 2, "subintervals_per_s": 1.9e13},  # impossible
        {"step": "riemann_parity_np3", "gpus": 3, "subintervals_per_s": 5e12},
        {"step": "miint_comm_np2", "op": "allreduce", "bytes": 8},
        {"step": "miint_comm_np2", "op": "allgather", "bytes": 16},
    ]
    path = tmp_path / "records.jsonl"
    path.write_text("".join(json.dumps(r) + "\n" for r in recs))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shared_rccl_report.py"),
                        str(path)], capture_output=True, text=True)
    assert p.returncode == 1, p.stdout + p.stderr
    rows = {l.split("|")[1].strip(): l for l in p.stdout.splitlines() if l.startswith("| ")}
    assert rows["riemann_np2"].rstrip().endswith("| yes |")
    assert "**NO**" in rows["miint_bench_np2"]
    assert "NET/Socket" in rows["riemann_np2"]
    assert p.stdout.count("miint_comm_np2") == 1  # one row per step
    assert "one-rank rate: 1" in p.stdout


def test_roofline_t2d_multistep_counts_the_replay(tmp_path):
    """A 2-D multi-step dispatch runs one replay of integrations (512 of 4096^2 since round 5,
    Table2DPlan::graph_steps): VALU per sample divides by all of them; a Riemann multi-step
    dispatch is not multiplied."""
    d = tmp_path / "table2d_G1"
    os.makedirs(d)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Correlation_Id", "Kernel_Name",
                                          "Counter_Name", "Counter_Value", "Start_Timestamp",
                                          "End_Timestamp"])
        w.writeheader()
        w.writerow({"Dispatch_Id": 1, "Correlation_Id": 1,
                    "Kernel_Name": "void miint::(anonymous namespace)::table2d_multistep_kernel<30>(x)",
                    "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 9.23e8,
                    "Start_Timestamp": 0, "End_Timestamp": 2_231_100})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline.py"),
                          str(tmp_path)], capture_output=True, text=True, check=True).stdout
    row = [ln for ln in out.splitlines() if ln.startswith("| table2d")][0]
    cells = [c.strip() for c in row.strip("|").split("|")]
    assert cells[4] == f"{9.23e8 * 64 / (4096 * 4096 * 512):.2f}" == "6.88"
