#!/usr/bin/env python3
"""Two ranks, one GPU: native RCCL communicator over a gloo process group.

Probes the multi-rank bootstrap on the 1-GPU pool. Run under torchrun --nproc-per-node 2.
Result on ROCm 7.2 (gpurun, 2026-10-15): both ranks exchange the unique id through the
torch store and reach ncclCommInitRank, which RCCL rejects with "invalid usage": two ranks
may not share a device. The 8-GPU node runs one GPU per rank. Multi-rank numerics are
covered by the gloo tests; the 1-rank RCCL graph path by test_plan_rccl_stage_on_one_gpu.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cuda_v_mpi_amd import Integrator  # noqa: E402
from cuda_v_mpi_amd.parallel import dist as mdist  # noqa: E402

ctx = mdist.init(backend="gloo")
it = Integrator("pi4", n=2 * 10**8, rule="mid", ctx=ctx, comm="native")
t = it.run_steps(33, pipeline=True, graphs=True)
vals = [it.plan.host_result(it.plan.host_index_of(k, True)) for k in range(17, 33)]
print(f"rank {ctx.rank}: bucketed={it.plan.bucketed} graphs={it.plan.graphs_ready} "
      f"value={vals[-1]!r} all_equal={len(set(vals)) == 1} device_ms={t['device_ms']:.3f}",
      flush=True)
ctx.barrier()
ctx.destroy()
