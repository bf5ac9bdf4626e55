"""Data fixtures: the 1801-sample train velocity profile (reference ``ex4vel.h``).

The reference ships the table as a 211-line C header "auto-generated from Excel"
(ex4vel.h:1-8). Its values live bit-exact in ONE place, csrc/runtime/profile_data.cpp
(hex-float literals, sha256 pinned as PROFILE_SHA256); this module reads them from that
file's text, so Python and the native runtime share the same bits without the extension.

The table is also the discrete form of a 7-phase jerk-limited profile:
``generated_profile_table()`` rebuilds it from that definition (running sums of a
piecewise-constant jerk of 0.002904762 m/s^3, rounded to 15 significant digits like the
spreadsheet export) and lands within 1.1e-13 of the data everywhere — an independent check
that the data is the profile it claims to be.
"""
from __future__ import annotations

import functools
import math
import os
import re

import numpy as np

PROFILE_LEN = 1801
PROFILE_SECONDS = 1800
STEPS_PER_SEC = 10000
JERK = 0.002904762

REFERENCE_HEADER = "/root/reference/ex4vel.h"
PROFILE_SHA256 = "4ebfbb500555fc9d7d054031eb7d9ec8cd813b71513480d569e2e4eee9b18a7a"
PROFILE_DATA_SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "csrc", "runtime", "profile_data.cpp")


def accel_steps(i: int) -> int:
    """Acceleration of second i in units of JERK (the 7 phases)."""
    if i < 100:
        return i + 1            # jerk +: 0 -> 0.2904762 m/s^2 over 100 s
    if i < 300:
        return 100              # constant acceleration
    if i < 399:
        return 399 - i          # jerk -
    if i < 1400:
        return 0                # cruise at 87.14286 m/s
    if i < 1499:
        return -(i - 1399)      # braking: jerk -
    if i < 1700:
        return -100             # constant deceleration
    if i < 1799:
        return -(1799 - i)      # jerk +
    return 0


def _round15(x: float) -> float:
    return float(f"{x:.15g}")


@functools.lru_cache(maxsize=1)
def _generated_tuple() -> tuple:
    v = [0.0] * PROFILE_LEN
    vel = acc = 0.0
    kprev = 0
    for i in range(PROFILE_SECONDS):
        k = accel_steps(i)
        acc = acc + float(k - kprev) * JERK
        kprev = k
        vel = vel + acc
        v[i + 1] = vel
    return tuple(_round15(x) for x in v)


@functools.lru_cache(maxsize=1)
def _profile_tuple() -> tuple:
    with open(PROFILE_DATA_SRC) as fh:
        src = fh.read()
    body = src[src.index("kProfileData[kProfileLen] = {") + 29:]
    body = body[:body.index("};")]
    vals = tuple(float.fromhex(t) for t in re.findall(r"-?0x[0-9a-fA-F.]+p[-+]?\d+", body))
    if len(vals) != PROFILE_LEN:
        raise ValueError(f"{PROFILE_DATA_SRC}: expected {PROFILE_LEN} values, got {len(vals)}")
    return vals


def profile_sha256(table: np.ndarray) -> str:
    import hashlib

    return hashlib.sha256(np.asarray(table, dtype="<f8").tobytes()).hexdigest()


def profile_table() -> np.ndarray:
    """DefaultProfile (float64[1801]), bit-exact; a fresh copy each call."""
    return np.array(_profile_tuple(), dtype=np.float64)


def generated_profile_table() -> np.ndarray:
    """The profile rebuilt from its 7-phase jerk definition (within 1.1e-13 of the data)."""
    return np.array(_generated_tuple(), dtype=np.float64)


def load_reference_table(path: str = REFERENCE_HEADER) -> np.ndarray | None:
    """Parse the reference header (text only) if it exists; None otherwise."""
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        s = fh.read()
    body = s[s.index("{") + 1:s.rindex("}")]
    vals = [float(t) for t in re.findall(r"[-+0-9.eE]+", body)]
    return np.array(vals, dtype=np.float64)


def interp(table: np.ndarray, t):
    """Vectorised linear interpolation with the segment index clamped to the table."""
    t = np.asarray(t, dtype=np.float64)
    i = np.clip(np.floor(t).astype(np.int64), 0, table.size - 2)
    fr = t - i
    return table[i] + (table[i + 1] - table[i]) * fr


def table_integral(a: float = 0.0, b: float = float(PROFILE_SECONDS)) -> float:
    """Exact integral of the piecewise-linear interpolant over [a, b] (0 <= a <= b <= 1800)."""
    v = _profile_tuple()

    def prim(t: float) -> float:
        i = int(min(max(math.floor(t), 0), PROFILE_LEN - 2))
        full = math.fsum(0.5 * (v[k] + v[k + 1]) for k in range(i))
        fr = t - i
        return full + fr * v[i] + 0.5 * fr * fr * (v[i + 1] - v[i])

    return prim(b) - prim(a)
