"""Integration steps driven through torch.distributed instead of the native communicator.

Each step launches the fused gfx950 Riemann kernel on the current torch stream, writing the
rank's partial into row k of a device tensor, and all-reduces that row with
torch.distributed (``nccl`` = RCCL on ROCm). ``async_op=True`` lets RCCL's internal stream
pick up step k while the kernel of step k+1 already runs on the compute stream.

This is the "one process per GPU with torch.distributed" form of the reference's
master/worker reduction (riemann.cpp:76-85); the native form (C++ RCCL communicator inside
a hipGraph) lives in csrc/runtime/integrator.cpp.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..models.integrands import IntegrandSpec
from ..ops import kernels
from .decomposition import rank_slice
from .dist import DistContext


class TorchStepper:
    def __init__(self, spec: IntegrandSpec, n_total: int, ctx: DistContext, rule: str = "left",
                 dtype: str = "fp64", div: str = "series_exact", grid: int | None = None,
                 capacity: int = 4096, group=None):
        self.spec, self.n, self.ctx = spec, int(n_total), ctx
        self.rule, self.dtype, self.div = rule, dtype, div
        self.begin, self.count = rank_slice(self.n, ctx.rank, ctx.world)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.ws = kernels.FusedWorkspace(grid or kernels.default_grid(), dev)
        self.out = torch.zeros(capacity, dtype=torch.float64, device=dev)
        self._works = []
        # None = the default process group (nccl, or gloo on CUDA tensors for ranks that
        # share a device); a gloo control-plane rank passes ctx.nccl_group()
        self.group = group

    def launch_steps(self, steps: int) -> None:
        self._works = []
        cap = self.out.numel()
        for k in range(steps):
            row = self.out[k % cap:k % cap + 1]
            if k >= cap and self.ctx.world > 1:
                # row k % cap is about to be overwritten: the compute stream first waits
                # for the all-reduce of step k - cap that still reads it
                self._works[k - cap].wait()
            kernels.riemann(self.spec, self.n, rule=self.rule, dtype=self.dtype, div=self.div,
                            i_begin=self.begin, n_local=self.count, out=row, workspace=self.ws)
            if self.ctx.world > 1:
                self._works.append(dist.all_reduce(row, group=self.group, async_op=True))

    def sync(self) -> None:
        for w in self._works:
            w.wait()
        self._works = []
        torch.cuda.synchronize()

    def result(self, k: int) -> float:
        return float(self.out[k % self.out.numel()].item())
