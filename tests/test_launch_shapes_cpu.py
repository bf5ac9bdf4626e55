"""Host-side launch-shape rules of the native kernels, checked without a GPU (the rules are
plain host code in the extension): which 2-D field kernel a grid runs and how many
workgroups it launches. The kernels themselves are checked on the GPU
(tests/test_gpu_kernels.py)."""
from __future__ import annotations

import pytest

F = 1801  # the profile table: 1801 x 1801 cells + 1


@pytest.mark.parametrize("g,rows,path,wgs", [
    (4096, (0, 4096), "stream", 16 * 64),   # 256 columns x 64 rows per workgroup (R = 16)
    (8192, (0, 8192), "stream", 32 * 64),   # R = 32: 256 x 128 fits at 8192^2
    (4096, (0, 512), "stream", 16 * 32),    # an 8-GPU slice: R = 4 keeps 512 workgroups
    (4096, (3584, 4096), "stream", 16 * 32),
    (2048, (0, 2048), "tile", 32 * 32),     # 0.88 cells per sample: 64-sample tiles
    (1000, (0, 1000), "tile", 16 * 16),
])
def test_table2d_shape(native, g, rows, path, wgs):
    args = (F, F, 1800.0, 1800.0, g, g, rows[0], rows[1])
    assert native.table2d_path(*args) == path
    assert native.table2d_grid(*args) == wgs


def test_table2d_stream_needs_fine_columns(native):
    # rows fine enough, columns too coarse for a 128-cell footprint -> tile kernel
    assert native.table2d_path(F, F, 1800.0, 1800.0, 3000, 8192, 0, 8192) == "tile"
    assert native.table2d_path(F, F, 1800.0, 1800.0, 8192, 3000, 0, 3000) == "stream"
