"""The 2-D row stream's LDS tile must hold every footprint it is given (kernels/table.hip
table2d_shape: a block of 4 R sample rows and 256 sample columns touches at most
floor((n - 1) step) + 3 table rows / columns). This checks the bound the shape selection uses
against every block's actual footprint — the kernel's own index formulas in fp64, as the
device evaluates them — over many grids, slices and shape targets, on the CPU (the shape
selection is host code in the extension; no GPU needed). A violation would be an LDS read
outside the staged tile (the GPU LDS-poison tests catch it only for the shapes they run)."""
from __future__ import annotations

import random

import pytest

from cuda_v_mpi_amd import native

WAVE, SCOLS = 64, 4


def _clampi(v, lo, hi):
    return max(lo, min(v, hi))


def _footprints(nx, ny, X, Y, gx, gy, row0, row1, rpw):
    """(max rows, max cols) of the table footprint over the launch's blocks."""
    sx, sy = X / gx, Y / gy
    cx, cy = (nx - 1) / X, (ny - 1) / Y
    rows = 0
    r0 = row0
    while r0 < row1:
        r1 = min(r0 + 4 * rpw, row1)
        ty0 = _clampi(int(((r0 + 0.5) * sy) * cy), 0, ny - 2)
        ty1 = _clampi(int(((r1 - 1 + 0.5) * sy) * cy), 0, ny - 2) + 1
        rows = max(rows, ty1 - ty0 + 1)
        r0 = r1
    cols = 0
    c0 = 0
    while c0 < gx:
        clast = min(c0 + WAVE * SCOLS, gx) - 1
        tx0 = _clampi(int(((c0 + 0.5) * sx) * cx), 0, nx - 2)
        tx1 = _clampi(int(((clast + 0.5) * sx) * cx), 0, nx - 2) + 1
        cols = max(cols, tx1 - tx0 + 1)
        c0 += WAVE * SCOLS
    return rows, cols


def _cases():
    rng = random.Random(20261017)
    out = [(1801, 4096, 1, 0, 0), (1801, 4096, 8, 0, 1), (1801, 4096, 8, 7, 1), (1801, 8192, 1, 0, 1),
           (1801, 5000, 8, 3, 0), (1801, 4095, 4, 0, 1), (1801, 6144, 2, 1, 1), (1801, 4097, 1, 0, 1)]
    for _ in range(60):
        n = rng.choice([1801, 901, 257, 4001])
        g = rng.randint(2 * n, 12000)
        w = rng.choice([1, 2, 4, 8, 16])
        out.append((n, g, w, rng.randrange(w), rng.choice([0, 1, 512, 2048])))
    return out


@pytest.mark.parametrize("n,g,w,r,min_wg", _cases())
def test_stream_tile_holds_every_footprint(n, g, w, r, min_wg):
    X = 1800.0
    base, rem = divmod(g, w)
    row0 = r * base + min(r, rem)
    row1 = row0 + base + (1 if r < rem else 0)
    info = native().table2d_shape_info(n, n, X, X, g, g, row0, row1, min_wg)
    if not info["stream"]:
        return
    rows, cols = _footprints(n, n, X, X, g, g, row0, row1, info["rows_per_wave"])
    assert rows <= info["tile_rows"], (info, rows)
    assert cols <= info["tile_cols"], (info, cols)
    # the staged window (SH whole rows from min(ty0, n - SH)) lies inside the table
    assert n >= info["tile_rows"]


def test_4096_shapes():
    """4096^2 with the multi-step plans' target (min_wg 1): 16 rows per wave, the 30-row tile,
    16 x 64 blocks; the 1/8 slice 16 x 8."""
    m = native()
    full = m.table2d_shape_info(1801, 1801, 1800.0, 1800.0, 4096, 4096, 0, 4096, 1)
    assert full["rows_per_wave"] == 16 and full["tile_rows"] == 30 and full["grid"] == (16, 64)
    s8 = m.table2d_shape_info(1801, 1801, 1800.0, 1800.0, 4096, 4096, 0, 512, 1)
    assert s8["rows_per_wave"] == 16 and s8["grid"] == (16, 8)


def test_auto_replay_steps_rule():
    """Table2DPlan's auto replay size (table2d_auto_graph_steps, host code): doubled from 32
    until a replay holds 2^33 samples of the LARGEST rank's rows, capped at 1024; 32 for a
    shape without the row stream (chained replays of one kernel node per integration). The
    same answer for every rank of an uneven split (it depends on grid and world only)."""
    m = native()
    assert m.table2d_auto_graph_steps(4096) == 512
    assert m.table2d_auto_graph_steps(4096, world=2) == 1024
    assert m.table2d_auto_graph_steps(4096, world=8) == 1024
    assert m.table2d_auto_graph_steps(4095, world=8) == 1024
    assert m.table2d_auto_graph_steps(8192) == 128
    assert m.table2d_auto_graph_steps(16384) == 32  # 2^28 samples x 32 = 2^33 already
    assert m.table2d_auto_graph_steps(1000) == 32   # the tile kernel
    assert m.table2d_auto_graph_steps(2048) == 32   # 0.88 table cells per sample: the tile kernel
    for g in (4096, 6144, 8192):  # row-stream shapes
        for w in (1, 2, 3, 4, 8):
            s = m.table2d_auto_graph_steps(g, world=w)
            rows = -(-g // w)
            assert s in (32, 64, 128, 256, 512, 1024)
            assert s == 1024 or s * g * rows >= 2**33
            assert s == 32 or (s // 2) * g * rows < 2**33
