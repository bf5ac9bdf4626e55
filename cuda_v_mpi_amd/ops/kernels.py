"""Tensor-level entry points to the gfx950 HIP kernels.

Every function takes/returns ``torch`` tensors on a HIP device and launches the native
kernel on the current torch stream (so it composes with torch.distributed collectives and
torch.cuda graphs). There is no fallback: a CPU tensor or a missing extension is an error.

Kernel sources: csrc/kernels/{riemann,table,scan,selftest}.hip.
"""
from __future__ import annotations

import math

import torch

from .._native import native
from ..models.integrands import IntegrandSpec

_RULE_OFF = {"left": 0.0, "mid": 0.5, "right": 1.0}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(t: torch.Tensor, dtype=torch.float64, name: str = "tensor") -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be on a HIP device (got {t.device})")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("HIP device required (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _enums(dtype: str, div: str):
    m = native()
    return getattr(m.DType, dtype), getattr(m.DivMode, div)


def default_grid() -> int:
    m = native()
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return m.default_riemann_grid(cus, 32)


def riemann_partials(spec: IntegrandSpec, n: int, rule: str = "left", dtype: str = "fp64",
                     div: str = "series_exact", grid: int | None = None, i_begin: int = 0,
                     n_local: int | None = None) -> torch.Tensor:
    """Per-workgroup unscaled partial sums of f over samples [i_begin, i_begin+n_local)."""
    m = native()
    dev = _device()
    grid = grid or default_grid()
    n_local = n if n_local is None else n_local
    h = (spec.b - spec.a) / n
    partials = torch.empty(grid, dtype=torch.float64, device=dev)
    table = _table_tensor(spec, dev)
    dt, dv = _enums(dtype, div)
    m.launch_riemann_partials(spec.native_id, spec.a, h, _RULE_OFF[rule], i_begin, n_local,
                              list(spec.coef), spec.p0, spec.p1, dt, dv, grid,
                              table.data_ptr() if table is not None else 0,
                              table.numel() if table is not None else 0,
                              partials.data_ptr(), _stream())
    return partials


_TABLE_CACHE: dict = {}


def _table_tensor(spec: IntegrandSpec, dev: torch.device):
    if spec.name != "table":
        return None
    key = (dev.index,)
    t = _TABLE_CACHE.get(key)
    if t is None:
        t = torch.tensor(spec.native_table(), dtype=torch.float64, device=dev)
        _TABLE_CACHE[key] = t
    return t


def finalize(partials: torch.Tensor, scale: float, out: torch.Tensor | None = None) -> torch.Tensor:
    _check(partials, name="partials")
    out = torch.empty(1, dtype=torch.float64, device=partials.device) if out is None else out
    native().launch_finalize(partials.data_ptr(), partials.numel(), scale, out.data_ptr(), _stream())
    return out


def unset_slots(n: int, device) -> torch.Tensor:
    """n fp64 write-once slots in their unset state (csrc/include/miint/handoff.hpp): what the
    one-launch reductions hand partials over in; the consuming workgroup re-arms them."""
    word = native().UNSET_SLOT_WORD
    bits = (word << 32) | word
    return torch.full((n,), bits - (1 << 64), dtype=torch.int64, device=device).view(torch.float64)


class FusedWorkspace:
    """Partials (write-once slots) + ticket for the one-launch reduction; reuse across
    calls (graph-safe: the kernel re-arms both)."""

    def __init__(self, grid: int, device: torch.device | None = None):
        dev = device or _device()
        self.grid = grid
        self.partials = unset_slots(grid, dev)
        self.ticket = torch.zeros(native().TICKET_WORDS, dtype=torch.int32, device=dev)


def riemann(spec: IntegrandSpec, n: int, rule: str = "left", dtype: str = "fp64",
            div: str = "series_exact", grid: int | None = None, i_begin: int = 0,
            n_local: int | None = None, out: torch.Tensor | None = None,
            workspace: FusedWorkspace | None = None, fused: bool = True) -> torch.Tensor:
    """h * scale * sum f over this launch's samples, as a 1-element fp64 device tensor."""
    m = native()
    dev = _device()
    grid = grid or (workspace.grid if workspace else default_grid())
    n_local = n if n_local is None else n_local
    h = (spec.b - spec.a) / n
    scale = h * spec.scale
    out = torch.empty(1, dtype=torch.float64, device=dev) if out is None else out
    if not fused:
        p = riemann_partials(spec, n, rule, dtype, div, grid, i_begin, n_local)
        return finalize(p, scale, out)
    ws = workspace or FusedWorkspace(grid, dev)
    table = _table_tensor(spec, dev)
    dt, dv = _enums(dtype, div)
    m.launch_riemann_fused(spec.native_id, spec.a, h, _RULE_OFF[rule], i_begin, n_local,
                           list(spec.coef), spec.p0, spec.p1, dt, dv, ws.grid,
                           table.data_ptr() if table is not None else 0,
                           table.numel() if table is not None else 0,
                           ws.partials.data_ptr(), ws.ticket.data_ptr(), scale, out.data_ptr(),
                           _stream())
    return out


def point_values(spec: IntegrandSpec, n: int, rule: str = "left", div: str = "series",
                 i_begin: int = 0, n_local: int | None = None) -> torch.Tensor:
    """Every sample's f value exactly as the hot tile path computes it (validation)."""
    m = native()
    dev = _device()
    n_local = n if n_local is None else n_local
    out = torch.empty(n_local, dtype=torch.float64, device=dev)
    table = _table_tensor(spec, dev)
    m.launch_riemann_point_values(spec.native_id, spec.a, (spec.b - spec.a) / n, _RULE_OFF[rule],
                                  i_begin, n_local, list(spec.coef), spec.p0, spec.p1,
                                  getattr(m.DivMode, div),
                                  table.data_ptr() if table is not None else 0,
                                  table.numel() if table is not None else 0,
                                  out.data_ptr(), _stream())
    return out


def pi4_recip_narrow(d: torch.Tensor) -> torch.Tensor:
    """The IEEE-division kIeee Pi4 tiles' reciprocal of every element of ``d`` (validation:
    bitwise 1 / d for 1 <= d <= 2**500 in fp64, 2**100 in fp32 — the fp32 tiles' form)."""
    f32 = d.dtype == torch.float32
    _check(d, dtype=torch.float32 if f32 else torch.float64, name="d")
    out = torch.empty_like(d)
    launch = native().launch_pi4_recip_narrow_f32 if f32 else native().launch_pi4_recip_narrow
    launch(d.data_ptr(), d.numel(), out.data_ptr(), _stream())
    return out


def sum_array(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    _check(x, name="x")
    m = native()
    cus = torch.cuda.get_device_properties(x.device).multi_processor_count
    grid = m.default_reduce_grid(cus)
    partials = torch.empty(grid, dtype=torch.float64, device=x.device)
    out = torch.empty(1, dtype=torch.float64, device=x.device)
    m.launch_sum_array(x.data_ptr(), x.numel(), scale, partials.data_ptr(), grid, out.data_ptr(),
                       _stream())
    return out


def profile_tensor(device=None) -> torch.Tensor:
    from ..models import integrands
    dev = device or _device()
    return _table_tensor(integrands.table(), torch.device(dev))


def interp_fill(n: int, i0: int = 0, dt: float = 1e-4, out: torch.Tensor | None = None) -> torch.Tensor:
    dev = _device()
    tab = profile_tensor(dev)
    out = torch.empty(n, dtype=torch.float64, device=dev) if out is None else out
    _check(out, name="out")
    native().launch_interp_fill(tab.data_ptr(), tab.numel(), dt, i0, n, out.data_ptr(), _stream())
    return out


def _scan_state(n: int, dev) -> torch.Tensor:
    nbytes = native().scan_state_bytes(n)
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)


def inclusive_scan(x: torch.Tensor, carry: torch.Tensor | None = None,
                   out: torch.Tensor | None = None) -> torch.Tensor:
    """Single-pass decoupled look-back inclusive scan (fp64)."""
    _check(x, name="x")
    out = torch.empty_like(x) if out is None else out
    st = _scan_state(x.numel(), x.device)
    native().launch_inclusive_scan(x.data_ptr(), out.data_ptr(), x.numel(), st.data_ptr(),
                                   carry.data_ptr() if carry is not None else 0, _stream())
    _check_timeout(st)
    return out


def interp_scan(n: int, i0: int = 0, dt: float = 1e-4, window: tuple[int, int] | None = None,
                carry: torch.Tensor | None = None) -> torch.Tensor:
    """inclusive_scan(interp(profile, (i0+i)*dt)) fused in one pass."""
    dev = _device()
    tab = profile_tensor(dev)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    st = _scan_state(n, dev)
    lo, hi = window if window is not None else (0, (1 << 64) - 1)
    native().launch_interp_scan(tab.data_ptr(), tab.numel(), dt, i0, n, lo, hi, out.data_ptr(),
                                st.data_ptr(), carry.data_ptr() if carry is not None else 0,
                                _stream())
    _check_timeout(st)
    return out


def trainscan(n: int, i0: int = 0, dt: float = 1e-4, window: tuple[int, int] | None = None,
              carries: torch.Tensor | None = None, algo: str = "fused"):
    """Two-phase scan of the interpolated profile (csrc/kernels/trainscan.hip).

    Returns (vel, pos, totals): vel = running sum of the samples, pos = running sum of vel,
    totals = {T1, T2} (the slice's sample sum and vel sum without carries). `carries`
    (2-element device tensor {C1, C2}) shifts the slice as if it followed earlier ranks
    (algo="fused" only). algo="onepass": single pass with a decoupled look-back."""
    if algo not in ("fused", "onepass"):
        raise ValueError("algo must be fused|onepass")
    if algo == "onepass" and carries is not None:
        raise ValueError("the one-pass scan takes no carries (single-GPU form)")
    m = native()
    dev = _device()
    tab = profile_tensor(dev)
    vel = torch.empty(n, dtype=torch.float64, device=dev)
    pos = torch.empty(n, dtype=torch.float64, device=dev)
    ws = torch.zeros(m.trainscan_workspace_bytes(n), dtype=torch.uint8, device=dev)  # zeroed once
    totals = torch.zeros(2, dtype=torch.float64, device=dev)
    lo, hi = window if window is not None else (0, (1 << 64) - 1)
    if algo == "onepass":
        m.launch_trainscan_onepass(tab.data_ptr(), tab.numel(), dt, i0, n, lo, hi, ws.data_ptr(),
                                   totals.data_ptr(), vel.data_ptr(), pos.data_ptr(), _stream())
        if m.trainscan_onepass_timeout(ws.data_ptr(), _stream()):
            raise RuntimeError("trainscan look-back spin limit hit")
        return vel, pos, totals
    m.launch_trainscan(tab.data_ptr(), tab.numel(), dt, i0, n, lo, hi, ws.data_ptr(),
                       totals.data_ptr(), carries.data_ptr() if carries is not None else 0,
                       vel.data_ptr(), pos.data_ptr(), _stream())
    return vel, pos, totals


def _check_timeout(state: torch.Tensor) -> None:
    flag = native().scan_timeout_flag(state.data_ptr(), _stream())
    if flag:
        raise RuntimeError("scan look-back spin limit hit (inter-workgroup hand-off failed)")


def add_carry(x: torch.Tensor, carry: torch.Tensor) -> torch.Tensor:
    _check(x, name="x")
    native().launch_add_carry(x.data_ptr(), x.numel(), carry.data_ptr(), _stream())
    return x


def outer_product(v: torch.Tensor) -> torch.Tensor:
    _check(v, name="v")
    n = v.numel()
    t = torch.empty((n, n), dtype=torch.float64, device=v.device)
    native().launch_outer_product(v.data_ptr(), n, t.data_ptr(), _stream())
    return t


def table2d(table: torch.Tensor, X: float, Y: float, gx: int, gy: int, row0: int = 0,
            row1: int | None = None, fused: bool = True) -> torch.Tensor:
    """Midpoint-rule integral of the bilinear interpolant of `table` (ny x nx) over
    [0,X]x[0,Y] on a gx x gy grid, sample rows [row0, row1) only. 1-element tensor.
    fused: one launch with the last-workgroup reduction; else partials + finalize."""
    _check(table, name="table")
    ny, nx = table.shape
    row1 = gy if row1 is None else row1
    m = native()
    grid = m.table2d_grid(nx, ny, X, Y, gx, gy, row0, row1)
    partials = (unset_slots(grid, table.device) if fused
                else torch.empty(grid, dtype=torch.float64, device=table.device))
    if not fused:
        m.launch_table2d_partials(table.data_ptr(), nx, ny, X, Y, gx, gy, row0, row1,
                                  partials.data_ptr(), _stream())
        return finalize(partials, 1.0)
    ticket = torch.zeros(m.TICKET_WORDS, dtype=torch.int32, device=table.device)
    out = torch.empty(1, dtype=torch.float64, device=table.device)
    m.launch_table2d_fused(table.data_ptr(), nx, ny, X, Y, gx, gy, row0, row1,
                           partials.data_ptr(), ticket.data_ptr(), out.data_ptr(), _stream())
    return out


def table2d_reference(table: torch.Tensor, X: float, Y: float, gx: int, gy: int,
                      row0: int = 0, row1: int | None = None, rows_per_chunk: int = 256) -> float:
    """Plain torch fp64 form of `table2d` (any device, CPU included): the same midpoint
    samples and bilinear blend, summed in row chunks of at most rows_per_chunk x gx."""
    ny, nx = table.shape
    row1 = gy if row1 is None else row1
    t = table.to(torch.float64)
    xs = (torch.arange(gx, dtype=torch.float64, device=t.device) + 0.5) * (X / gx) * ((nx - 1) / X)
    ix = xs.long().clamp(0, nx - 2)
    fx = (xs - ix).unsqueeze(0)
    total = 0.0
    for r in range(row0, row1, rows_per_chunk):
        rows = torch.arange(r, min(r + rows_per_chunk, row1), dtype=torch.float64, device=t.device)
        ys = (rows + 0.5) * (Y / gy) * ((ny - 1) / Y)
        iy = ys.long().clamp(0, ny - 2)
        fy = (ys - iy).unsqueeze(1)
        lo, hi = t[iy], t[iy + 1]
        top = lo[:, ix] + (lo[:, ix + 1] - lo[:, ix]) * fx
        bot = hi[:, ix] + (hi[:, ix + 1] - hi[:, ix]) * fx
        total += float((top + (bot - top) * fy).sum())
    return total * (X / gx) * (Y / gy)


def wave_ops(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(per-wave sums, per-wave inclusive scans) via the DPP primitives."""
    f32 = x.dtype == torch.float32
    _check(x, dtype=x.dtype, name="x")
    if x.dtype not in (torch.float32, torch.float64):
        raise ValueError("wave_ops supports fp32/fp64")
    sums = torch.empty(math.ceil(x.numel() / 64), dtype=x.dtype, device=x.device)
    scan = torch.empty_like(x)
    native().selftest_wave_ops(x.data_ptr(), x.numel(), f32, sums.data_ptr(), scan.data_ptr(),
                               _stream())
    return sums, scan


def block_ops(x: torch.Tensor, block: int) -> tuple[torch.Tensor, torch.Tensor]:
    f32 = x.dtype == torch.float32
    _check(x, dtype=x.dtype, name="x")
    sums = torch.empty(math.ceil(x.numel() / block), dtype=x.dtype, device=x.device)
    scan = torch.empty_like(x)
    native().selftest_block_ops(x.data_ptr(), x.numel(), block, f32, sums.data_ptr(),
                                scan.data_ptr(), _stream())
    return sums, scan


_EXPR_CACHE: dict = {}


def riemann_expr(expr: str, a: float, b: float, n: int, rule: str = "left",
                 i_begin: int = 0, n_local: int | None = None) -> float:
    """Riemann sum of any f(x) given as one C++ expression over ``x`` (HIP device math:
    ``"exp(-x*x)"``, ``"sin(x)/x"``, ...), compiled for gfx950 at run time with hipRTC
    (csrc/runtime/expr.cpp) and cached per (expression, device). Every sample is evaluated
    in fp64; the value is h * sum over samples [i_begin, i_begin + n_local) of the n-sample
    rule on [a, b]. The reference hard-wires sin (riemann.cpp:37) and recompiles to change it.
    """
    m = native()
    dev = _device().index
    key = (expr, dev)
    ei = _EXPR_CACHE.get(key)
    if ei is None:
        ei = _EXPR_CACHE[key] = m.ExprIntegrator(expr, dev)
    n_local = n - i_begin if n_local is None else n_local
    return ei.integrate(float(a), float(b), int(n), getattr(m.Rule, rule), int(i_begin),
                        int(n_local))
