"""cuda_v_mpi_amd — an MI355X-native numerical-integration framework.

Capabilities of the reference (Excalibur1224/Cuda-v-MPI: riemann.cpp, cintegrate.cu,
4main.c, ex4vel.h), rebuilt for AMD Instinct MI355X (gfx950 / CDNA4):

  * Riemann sums of sin(x), 4/(1+x^2), random polynomials and the analytic train model,
    fp64 and packed-fp32, as hand-written HIP kernels with wave64 DPP + LDS reductions;
  * train-profile integration: LDS-staged interpolation of the 1801-point velocity table,
    fused sums, and a single-pass decoupled look-back prefix scan;
  * multi-GPU: one process per GPU, RCCL all-reduce / all-gather over xGMI, hipGraph replay;
  * the reference's CLIs and stdout format (build/bin/{riemann,cintegrate,trainscan,miint}
    and ``python -m cuda_v_mpi_amd``), with --parity emulation of its partition arithmetic;
  * the reference's CPU (MPI) side, native: per-ISA vector kernels on host threads, host
    ranks with rank-order TCP collectives (``backend="host"``, ``--device cpu``,
    ``python -m cuda_v_mpi_amd compare``);
  * any integrand at run time: one C++ expression over x compiled for gfx950 with hipRTC
    (``ops.kernels.riemann_expr``, ``riemann --expr``).

Layout: models/ (integrands), ops/ (kernel entry points), parallel/ (decomposition,
process groups), utils/ (fixtures, oracles, output formats), integrate.py (high-level API).
"""
from __future__ import annotations

__version__ = "0.1.0"

from ._native import native, require_gpu  # noqa: F401
from .integrate import IntegrationResult, Integrator, integrate, integrate_expr  # noqa: F401
from .models import integrands  # noqa: F401
