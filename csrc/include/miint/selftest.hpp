// Self-test entry points for the wave64 DPP primitives (see kernels/selftest.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace miint {

// Per-wave sums (ceil(n/64) outputs) and per-wave inclusive scans (n outputs).
void selftest_wave_ops(const void* in, uint64_t n, bool f32, void* sums, void* scan,
                       hipStream_t s);
// Per-workgroup sums (ceil(n/block)) and per-workgroup inclusive scans (n outputs).
void selftest_block_ops(const void* in, uint64_t n, int block, bool f32, void* sums, void* scan,
                        hipStream_t s);

}  // namespace miint
