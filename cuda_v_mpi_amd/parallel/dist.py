"""Process-group bootstrap: one process per GPU under torchrun / torch.distributed.

Replaces MPI_Init/Comm_size/Comm_rank (riemann.cpp:62-64, 4main.c:69-71). Two kinds of
communicator come out of it:
  * the torch.distributed process group (backend "nccl" == RCCL on ROCm, "gloo" on CPU);
  * a native RCCL communicator owned by the C++ runtime (``_miint.Comm``), bootstrapped with
    a unique id that rank 0 publishes through the torch.distributed store. The native one is
    what the Riemann plans capture into hipGraphs together with their kernels.

A rank whose data plane is the native communicator keeps ONE RCCL communicator: its torch
process group is gloo (``control_backend``), which carries only the control plane (flags,
scalar gathers, barriers) on host tensors. A torch RCCL group is created only on demand
(``DistContext.nccl_group``: the torch.distributed step path) and counted in
``DistContext.nccl_groups`` so a run record can show how many the rank built.
"""
from __future__ import annotations

import dataclasses
import datetime
import os

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: int = 0
    backend: str = "none"
    initialized_here: bool = False
    nccl_groups: int = 0  # torch RCCL process groups this rank created (default one included)
    _nccl: object = None

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def host_collectives(self) -> bool:
        """Control-plane collectives take host tensors (gloo) rather than device ones."""
        return self.backend != "nccl"

    def control_device(self) -> str:
        return "cpu" if self.host_collectives else "cuda"

    def nccl_group(self):
        """The torch RCCL group for device-tensor collectives: the default group when it is
        nccl, else one created here on first use (every rank must call this together)."""
        if self.world == 1 or self.backend == "nccl":
            return None  # default group
        if self._nccl is None:
            self._nccl = dist.new_group(backend="nccl")
            self.nccl_groups += 1
        return self._nccl

    def barrier(self) -> None:
        if self.world > 1 and dist.is_initialized():
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device])
            else:
                dist.barrier()

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t

    def all_gather_scalars(self, value: float, device=None) -> list[float]:
        dev = device if device is not None else ("cuda" if self.backend == "nccl" else "cpu")
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        if self.world == 1:
            return [value]
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [float(x.item()) for x in out]

    def destroy(self) -> None:
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized_here = False


def ranks_share_devices() -> bool:
    """MIINT_OVERSUBSCRIBE=1: more ranks than GPUs (W ranks on a one-GPU box). The native
    runtime reads the same variable (``miint::ranks_share_devices``, comm.hpp)."""
    return os.environ.get("MIINT_OVERSUBSCRIBE", "") not in ("", "0")


def prepare_shared_device_rccl(rank: int) -> None:
    """RCCL refuses two ranks of one host on one GPU, so under ``ranks_share_devices`` each
    rank names itself a host of its own and the ranks meet over RCCL's socket transport on
    loopback: the multi-rank RCCL path runs for real, at socket speed (a correctness
    configuration). Mirrors ``miint::prepare_shared_device_rccl`` for torch's RCCL groups."""
    if not ranks_share_devices():
        return
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ["NCCL_HOSTID"] = f"miint-shared-rank-{rank}"


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str | None = None, timeout_s: float = 300.0, force: bool = False) -> DistContext:
    """Initialise from the torchrun environment (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    Single-process runs skip process-group creation unless ``force``. The default
    MASTER_ADDR is 127.0.0.1 (the container hostname may not resolve).
    """
    rank, world, local = env_world()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    ctx = DistContext(rank=rank, world=world, local_rank=local, backend=backend)
    prepare_shared_device_rccl(rank)
    if backend == "nccl":
        ctx.device = local % torch.cuda.device_count() if ranks_share_devices() else local
        torch.cuda.set_device(ctx.device)
    elif torch.cuda.is_available():
        # gloo process group with GPU compute: ranks may share devices (testing on 1 GPU)
        ctx.device = local % torch.cuda.device_count()
        torch.cuda.set_device(ctx.device)
    if world > 1 or force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", ctx.device)
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            ctx.initialized_here = True
            ctx.nccl_groups = int(backend == "nccl")
    else:
        ctx.backend = backend if dist.is_initialized() else "none"
    return ctx


def control_backend(data_plane: str, device: str = "gpu") -> str:
    """Process-group backend for a rank whose collectives go through ``data_plane``.

    ``native``: the C++ RCCL communicator carries every device collective, so the torch group
    is gloo (control plane only: one RCCL communicator per rank, not two). ``torch``: the
    torch group itself is the data plane, nccl on a GPU. CPU runs are gloo either way."""
    if device == "cpu":
        return "gloo"
    return "gloo" if data_plane == "native" else "nccl"


_uid_counter = [0]


def native_comm(ctx: DistContext):
    """Create a native RCCL communicator (``_miint.Comm``) spanning the process group."""
    from .._native import native

    m = native()
    _uid_counter[0] += 1
    if ctx.world == 1:
        return m.Comm(m.Comm.unique_id(), 0, 1, ctx.device)
    store = dist.distributed_c10d._get_default_store()
    key = f"miint_rccl_uid_{_uid_counter[0]}"
    if ctx.rank == 0:
        store.set(key, m.Comm.unique_id())
    uid = store.get(key)
    return m.Comm(bytes(uid), ctx.rank, ctx.world, ctx.device)
