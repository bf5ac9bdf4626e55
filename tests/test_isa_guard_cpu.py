"""ISA / resource regression guard (tools/isa_guard.py) on the CPU box: the hot gfx950
kernels are compiled device-only to assembly and compared with tools/isa_baseline.json —
hot-loop VALU (+3 % fails), scratch, waves per SIMD. The per-sample loop these kernels
replace is riemann.cpp:34-41; their speed rests on the exact allocation pinned here."""
from __future__ import annotations

import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import isa_guard  # noqa: E402


@pytest.fixture(scope="module")
def measured():
    if not os.path.exists(isa_guard.HIPCC):
        pytest.skip("hipcc not available")
    return isa_guard.measure()


def test_baseline_covers_every_guarded_kernel():
    with open(isa_guard.BASELINE) as f:
        base = json.load(f)
    assert set(base) == set(isa_guard.GUARDED)
    for k, v in base.items():
        assert "missing" not in v, k
        assert v["occupancy"] >= 4 and v["hot_loop_valu"] > 0, k


def test_no_isa_regression(measured):
    with open(isa_guard.BASELINE) as f:
        base = json.load(f)
    assert isa_guard.compare(base, measured) == []


def test_headline_kernel_shape(measured):
    """The headline kernels: the multi-step series_exact launch the bench runs (7 waves per
    SIMD, no scratch, one 384-sample tile's straight line <= 2.65 VALU per sample:
    integrands.hpp Pi4, 1014 per tile) and the single-launch tiles (>= 7 waves per SIMD,
    <= 2.65 VALU per sample: 1007 / 1013 per 384 samples)."""
    ms = measured["ms_pi4_series_exact"]
    assert ms["occupancy"] >= 7 and ms["scratch"] == 0 and ms["vgpr"] <= 64
    assert ms["max_block_valu"] / 384 <= 2.65
    for name in ("pi4_series", "pi4_series_exact"):
        k = measured[name]
        assert k["occupancy"] >= 7 and k["scratch"] == 0
        assert k["valu_per_sample"] <= 2.65


def test_guard_flags_a_regression():
    base = {"k": {"occupancy": 8, "scratch": 0, "hot_loop_valu": 100,
                  "hot_loop_scratch_ops": 0, "max_block_valu": 50}}
    ok = {"k": {"occupancy": 8, "scratch": 0, "hot_loop_valu": 103, "hot_loop_scratch_ops": 0,
                "max_block_valu": 51}}
    assert isa_guard.compare(base, ok) == []
    for bad in ({"hot_loop_valu": 104}, {"occupancy": 7}, {"scratch": 16},
                {"hot_loop_scratch_ops": 2}, {"max_block_valu": 52}):
        now = {"k": dict(ok["k"], **bad)}
        assert len(isa_guard.compare(base, now)) == 1, bad


def test_loops_are_natural_loops():
    """A loop closed by an unconditional latch counts; a backward jump of the block layout
    that re-enters code before a loop (no dominating target) does not."""
    body = "\n".join([
        "  s_cmp_eq_u32 s0, 0",
        "  s_cbranch_scc1 .LBB0_4",   # entry -> 4 (a block laid out after the loop)
        ".LBB0_1:",
        "  v_add_f64 v[0:1], v[0:1], v[2:3]",
        ".LBB0_2:",                   # loop: 2 -> 3 -> 2 (unconditional latch)
        "  v_fma_f64 v[0:1], v[0:1], v[2:3], v[4:5]",
        "  v_fma_f64 v[0:1], v[0:1], v[2:3], v[4:5]",
        "  s_add_u32 s1, s1, -1",
        "  s_cbranch_scc0 .LBB0_5",
        ".LBB0_3:",
        "  v_mul_f64 v[0:1], v[0:1], v[2:3]",
        "  s_branch .LBB0_2",
        ".LBB0_4:",
        "  v_mov_b32 v0, 0",
        "  s_branch .LBB0_1",          # layout jump back: 1 does not dominate 4
        ".LBB0_5:",
        "  s_endpgm",
    ])
    found = [sum(1 for s in lp if s.startswith("v_")) for lp in isa_guard.loops(body)]
    assert found == [3]
