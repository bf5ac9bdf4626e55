"""Integrand "models": the workloads the framework integrates.

The reference's workloads are
  * ``sin(x)`` on [0, pi]                          riemann.cpp:37, cintegrate.cu:68
  * the linearly interpolated 1801-point velocity profile on [0, 1800]
                                                     cintegrate.cu:23-44, 4main.c:249-269
  * the analytic train model v(t) = (1 - cos(t/ts)) vs   riemann.cpp:103-116 (dead code there)
and BASELINE.json adds 4/(1+x^2) on [0, 1] (pi) and random-coefficient polynomials.

Each spec knows its native id, default domain, analytic value and a plain-PyTorch fp64
evaluation used as the numerics reference in tests and by the CPU backend.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Sequence

import numpy as np

from ..utils import fixtures

TRAIN_TS = 286.4788975   # riemann.cpp:7
TRAIN_AS = 0.2365890     # riemann.cpp:8
TRAIN_VS = 67.7777777    # riemann.cpp:9

NATIVE_ID = {"pi4": 0, "sin": 1, "poly": 2, "train": 3, "table": 4}


@dataclasses.dataclass(frozen=True)
class IntegrandSpec:
    name: str
    a: float
    b: float
    coef: tuple = ()
    p0: float = 0.0
    p1: float = 0.0

    @property
    def native_id(self) -> int:
        return NATIVE_ID[self.name]

    @property
    def scale(self) -> float:
        return 4.0 if self.name == "pi4" else 1.0

    # ------------------------------------------------------------------ analytic value
    def analytic(self, a: float | None = None, b: float | None = None) -> float:
        a = self.a if a is None else a
        b = self.b if b is None else b
        if self.name == "pi4":
            return 4.0 * (math.atan(b) - math.atan(a))
        if self.name == "sin":
            return math.cos(a) - math.cos(b)
        if self.name == "poly":
            return sum(c * (b ** (k + 1) - a ** (k + 1)) / (k + 1) for k, c in enumerate(self.coef))
        if self.name == "train":
            ts, vs = self.p0, self.p1
            return vs * ((b - ts * math.sin(b / ts)) - (a - ts * math.sin(a / ts)))
        if self.name == "table":
            return fixtures.table_integral(a, b)
        raise ValueError(self.name)

    # ------------------------------------------------------------------ reference f(x)
    def f_torch(self, x):
        """fp64 PyTorch evaluation (reference for kernel numerics tests)."""
        import torch

        x = x.to(torch.float64)
        if self.name == "pi4":
            return 4.0 / (1.0 + x * x)
        if self.name == "sin":
            return torch.sin(x)
        if self.name == "poly":
            y = torch.zeros_like(x)
            for c in reversed(self.coef):
                y = y * x + c
            return y
        if self.name == "train":
            return (1.0 - torch.cos(x / self.p0)) * self.p1
        if self.name == "table":
            tab = torch.as_tensor(fixtures.profile_table(), dtype=torch.float64, device=x.device)
            i = torch.clamp(x.floor().to(torch.int64), 0, tab.numel() - 2)
            fr = x - i.to(torch.float64)
            v0 = tab[i]
            return v0 + (tab[i + 1] - v0) * fr
        raise ValueError(self.name)

    def native_table(self) -> list:
        return list(fixtures.profile_table()) if self.name == "table" else []


def pi4() -> IntegrandSpec:
    return IntegrandSpec("pi4", 0.0, 1.0)


def sin() -> IntegrandSpec:
    return IntegrandSpec("sin", 0.0, math.pi)


def train() -> IntegrandSpec:
    return IntegrandSpec("train", 0.0, 1800.0, p0=TRAIN_TS, p1=TRAIN_VS)


def table() -> IntegrandSpec:
    return IntegrandSpec("table", 0.0, 1800.0)


def poly(coef: Sequence[float] | None = None, degree: int = 6, seed: int = 0,
         a: float = 0.0, b: float = 1.0) -> IntegrandSpec:
    """Random-init polynomial (BASELINE.json "synthetic integrands / random-init coefficients")."""
    if coef is None:
        rng = np.random.default_rng(seed)
        coef = rng.uniform(-1.0, 1.0, size=degree + 1).tolist()
    if not 1 <= len(coef) <= 16:
        raise ValueError("poly supports 1..16 coefficients")
    return IntegrandSpec("poly", a, b, coef=tuple(float(c) for c in coef))


REGISTRY = {"pi4": pi4, "sin": sin, "train": train, "table": table, "poly": poly}


def get(name: str, **kw) -> IntegrandSpec:
    try:
        return REGISTRY[name](**kw)
    except KeyError:
        raise ValueError(f"unknown integrand {name!r}; choose from {sorted(REGISTRY)}") from None
