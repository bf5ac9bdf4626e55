"""High-level integration API.

    >>> from cuda_v_mpi_amd import Integrator
    >>> r = Integrator("pi4", n=10**9).run()          # one MI355X, fp64, left rule
    >>> r.value, r.abs_err, r.subintervals_per_s

Backends
  ``hip``  the native runtime: gfx950 kernels, hipGraph replay, RCCL for world > 1
           (``comm="native"``: C++ RCCL communicator captured in the graph, default;
           ``comm="torch"``: kernels on the torch stream + torch.distributed all_reduce;
           ``comm_obj=``: any native communicator, e.g. a loopback rank, see
           parallel/loopback.py)
  ``host`` the native host engine (miint/host.hpp): the rank's slice evaluated per sample
           in fp64 on ``threads`` vector threads (AVX-512 / AVX2 / baseline, picked at run
           time), world > 1 reduced with torch.distributed (gloo). The reference's own (MPI,
           CPU) side of its CUDA-vs-MPI comparison; needs no GPU.
  ``cpu``  plain PyTorch fp64 evaluation of the rank's slice + torch.distributed (gloo)
           all_reduce. Exists so the decomposition / collective logic can be exercised
           without a GPU; it is never used implicitly.
"""
from __future__ import annotations

import dataclasses
import math
import time

import torch

from .models import integrands
from .parallel import decomposition
from .parallel.dist import DistContext, native_comm


@dataclasses.dataclass
class IntegrationResult:
    value: float
    analytic: float
    n: int
    integrand: str
    rule: str
    dtype: str
    gpus: int
    seconds_wall: float
    seconds_device: float

    @property
    def abs_err(self) -> float:
        return abs(self.value - self.analytic)

    @property
    def rel_err(self) -> float:
        return self.abs_err / abs(self.analytic) if self.analytic else float("nan")

    @property
    def subintervals_per_s(self) -> float:
        t = self.seconds_device if self.seconds_device > 0 else self.seconds_wall
        return self.n / t if t > 0 else float("nan")

    def as_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d.update(abs_err=self.abs_err, rel_err=self.rel_err,
                 subintervals_per_s=self.subintervals_per_s)
        return d


class Integrator:
    def __init__(self, integrand: str | integrands.IntegrandSpec = "pi4", n: int = 10**9,
                 rule: str = "left", dtype: str = "fp64", div: str = "series_exact",
                 backend: str = "hip", ctx: DistContext | None = None, comm: str = "native",
                 fused: bool = True, grid: int = 0, slots: int = 16, a: float | None = None,
                 b: float | None = None, force_collective: bool = False, bucket: bool = True,
                 chain: bool = True, comm_obj=None, threads: int = 0,
                 slice_of: tuple[int, int] | None = None, step_streams: int = 0,
                 block: int = 256, multistep: bool = True, close: str = "auto",
                 allreduce_to_host: bool = True, timeout_s: float = 300.0, **spec_kw):
        spec = integrands.get(integrand, **spec_kw) if isinstance(integrand, str) else integrand
        if a is not None or b is not None:
            spec = dataclasses.replace(spec, a=spec.a if a is None else a,
                                       b=spec.b if b is None else b)
        if n < 1:
            raise ValueError("n must be >= 1")
        if rule not in ("left", "mid", "right"):
            raise ValueError("rule must be left|mid|right")
        if dtype not in ("fp64", "fp32", "fp32acc"):
            raise ValueError("dtype must be fp64|fp32|fp32acc")
        self.spec, self.n, self.rule, self.dtype, self.div = spec, int(n), rule, dtype, div
        self.backend, self.comm_kind = backend, comm
        if comm_obj is not None:  # an existing native communicator (e.g. a loopback rank)
            ctx = DistContext(rank=comm_obj.rank, world=comm_obj.world, device=comm_obj.device,
                              backend=comm_obj.kind)
        self.ctx = ctx or DistContext()
        self.begin, self.count = decomposition.rank_slice(self.n, self.ctx.rank, self.ctx.world)
        self._plan = None
        self._comm = None
        self._pool = None
        if backend in ("hip", "host"):
            from ._native import native

            m = native()
            if backend == "hip" and m.device_count() < 1:
                raise RuntimeError("backend='hip' needs a HIP device; use backend='host' or "
                                   "'cpu' explicitly")
            cfg = m.RiemannConfig()
            cfg.integrand = getattr(m.Integrand, spec.name)
            cfg.a, cfg.b, cfg.n = spec.a, spec.b, self.n
            cfg.rule = getattr(m.Rule, rule)
            cfg.dtype = getattr(m.DType, dtype)
            cfg.div = getattr(m.DivMode, div)
            cfg.coef = list(spec.coef)
            cfg.p0, cfg.p1 = spec.p0, spec.p1
            cfg.table = spec.native_table()
            cfg.grid, cfg.fused, cfg.slots = grid, fused, slots
            cfg.block = block  # threads per workgroup (the reference's SP): 64 .. 1024
            cfg.force_collective = force_collective
            cfg.bucket = bucket
            cfg.chain = chain
            cfg.step_streams = step_streams
            cfg.multistep = multistep  # graph batches as one persistent launch
            cfg.close = close  # multi-step batches closed by a kernel or inside the launch
            cfg.allreduce_to_host = allreduce_to_host  # bucketed all-reduce into pinned memory
            cfg.timeout_s = timeout_s  # collective watchdog of the plan's sync (<= 0: none)
            if slice_of is not None:  # (rank, world): that rank's share, on this device
                cfg.slice_rank, cfg.slice_world = int(slice_of[0]), int(slice_of[1])
            self._m = m
            if backend == "host":
                self._cfg = cfg
                self._pool = m.HostPool(threads)
                return
            if comm_obj is not None:
                self._comm = comm_obj
                self._plan = m.RiemannPlan(cfg, comm_obj.device, comm_obj)
            elif (self.ctx.world > 1 or force_collective) and comm == "native":
                self._comm = native_comm(self.ctx)
                self._plan = m.RiemannPlan(cfg, self.ctx.device, self._comm)
            else:
                cfg.rank, cfg.world = self.ctx.rank, self.ctx.world
                self._plan = m.RiemannPlan(cfg, self.ctx.device)
        elif backend != "cpu":
            raise ValueError("backend must be 'hip', 'host' or 'cpu'")

    # ------------------------------------------------------------------ info
    @property
    def plan(self):
        return self._plan

    @property
    def h(self) -> float:
        return (self.spec.b - self.spec.a) / self.n

    def describe(self) -> dict:
        d = dict(integrand=self.spec.name, n=self.n, rule=self.rule, dtype=self.dtype,
                 backend=self.backend, rank=self.ctx.rank, world=self.ctx.world,
                 begin=self.begin, count=self.count)
        if self._plan is not None:
            d.update(grid=self._plan.grid, block=self._plan.block,
                     div=str(self._plan.effective_div).split(".")[-1])
        return d

    # ------------------------------------------------------------------ execution
    def _torch_reduce(self, value: float) -> float:
        dev = "cuda" if self.ctx.backend == "nccl" else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        self.ctx.all_reduce_sum(t)
        return float(t.item())

    def _cpu_local(self) -> float:
        spec, h = self.spec, self.h
        off = {"left": 0.0, "mid": 0.5, "right": 1.0}[self.rule]
        dt = torch.float64 if self.dtype == "fp64" else torch.float32
        chunk = 1 << 22
        parts = []
        for s in range(self.begin, self.begin + self.count, chunk):
            i = torch.arange(s, min(self.begin + self.count, s + chunk), dtype=torch.float64)
            x = (spec.a + (i + off) * h).to(dt)
            parts.append(float(spec.f_torch(x).to(torch.float64).sum()))
        return math.fsum(parts) * h

    def run(self) -> IntegrationResult:
        t0 = time.perf_counter()
        dev_s = 0.0
        if self.backend == "cpu":
            value = self._torch_reduce(self._cpu_local()) if self.ctx.world > 1 else self._cpu_local()
        elif self.backend == "host":
            t = time.perf_counter()
            value = self._m.host_riemann(self._cfg, self.begin, self.count, self._pool)
            dev_s = time.perf_counter() - t  # the rank's compute time ("device" = host cores)
            if self.ctx.world > 1:
                value = self._torch_reduce(value)
        else:
            if self._comm is not None or self.ctx.world == 1:
                t = self._plan.run_steps(1, pipeline=False, graphs=False)
                value = self._plan.host_result(0)
                dev_s = t["device_ms"] * 1e-3
            else:  # torch.distributed reduction of the native plan's local value
                t = self._plan.run_steps(1, pipeline=False, graphs=False)
                value = self._torch_reduce(self._plan.host_result(0))
                dev_s = t["device_ms"] * 1e-3
        wall = time.perf_counter() - t0
        return IntegrationResult(value=value, analytic=self.spec.analytic(), n=self.n,
                                 integrand=self.spec.name, rule=self.rule, dtype=self.dtype,
                                 gpus=self.ctx.world, seconds_wall=wall, seconds_device=dev_s)

    def run_steps(self, steps: int, pipeline: bool = True, graphs: bool = True) -> dict:
        """Back-to-back integrations on the native runtime (benchmark inner loop)."""
        if self._plan is None:
            raise RuntimeError("run_steps needs backend='hip'")
        return self._plan.run_steps(steps, pipeline, graphs)

    def launch_steps(self, steps: int, pipeline: bool = True, graphs: bool = True) -> None:
        if self._plan is None:
            raise RuntimeError("launch_steps needs backend='hip'")
        self._plan.launch_steps(steps, pipeline, graphs)

    def sync(self) -> None:
        if self._plan is not None:
            self._plan.sync()


def integrate(integrand: str = "pi4", n: int = 10**9, **kw) -> IntegrationResult:
    return Integrator(integrand, n=n, **kw).run()


def integrate_expr(expr: str, a: float, b: float, n: int = 10**9, rule: str = "left",
                   backend: str = "hip", ctx: DistContext | None = None, threads: int = 0,
                   analytic: float | None = None) -> IntegrationResult:
    """Integrate any f(x) given as one C++ expression over ``x`` (``"exp(-x*x)"``): compiled
    for gfx950 with hipRTC (``backend="hip"``) or for the host cores (``backend="host"``),
    this rank's slice of the n-sample rule evaluated per sample in fp64, world > 1 reduced
    with torch.distributed. ``analytic`` (if known) sets the result's error reference.
    """
    from ._native import native

    if rule not in ("left", "mid", "right"):
        raise ValueError("rule must be left|mid|right")
    m = native()
    ctx = ctx or DistContext()
    begin, count = decomposition.rank_slice(int(n), ctx.rank, ctx.world)
    rl = getattr(m.Rule, rule)
    t0 = time.perf_counter()
    if backend == "hip":
        value = m.ExprIntegrator(expr, ctx.device).integrate(float(a), float(b), int(n), rl,
                                                              begin, count)
    elif backend == "host":
        value = m.HostExpr(expr).integrate(float(a), float(b), int(n), rl, begin, count,
                                           m.HostPool(threads))
    else:
        raise ValueError("integrate_expr backend must be 'hip' or 'host'")
    dev_s = time.perf_counter() - t0
    if ctx.world > 1:
        dev = "cuda" if ctx.backend == "nccl" else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        ctx.all_reduce_sum(t)
        value = float(t.item())
    return IntegrationResult(value=value, analytic=float("nan") if analytic is None else analytic,
                             n=int(n), integrand=f"expr:{expr}", rule=rule, dtype="fp64",
                             gpus=ctx.world, seconds_wall=time.perf_counter() - t0,
                             seconds_device=dev_s)
