"""Tensor-level entry points to the gfx950 HIP kernels (csrc/kernels/*.hip)."""
from . import kernels  # noqa: F401
