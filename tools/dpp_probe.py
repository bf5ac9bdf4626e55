#!/usr/bin/env python3
"""Launch the DPP wave/block reduction self-test kernels on a large array (profiling probe).

Used by tools/profile_counters.sh to show, with PMC counters, that the wave64 reduction is
pure VALU/DPP (no LDS instructions) and that the block reduction touches LDS once per wave.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_v_mpi_amd.ops import kernels  # noqa: E402

x = torch.randn(1 << 24, dtype=torch.float64, device="cuda")
for _ in range(3):
    kernels.wave_ops(x)
    kernels.block_ops(x, 256)
    kernels.block_ops(x, 1024)
torch.cuda.synchronize()
print("dpp probe done")
