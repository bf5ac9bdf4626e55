// Last-workgroup hand-off for one-launch reductions (Riemann fused kernel, 2-D field).
//
// Every workgroup publishes its partial with an agent-scope (sc1, write-through) store,
// drains it (s_waitcnt vmcnt(0)), then takes a ticket with an agent-scope atomic. The
// workgroup that draws the last ticket acquires (agent fence: buffer_inv sc1) and reduces
// all partials in index order with sc1 loads — the R1 hand-off of cdna_hip_programming.md
// §6 G16. Placement-independent: correctness never depends on which XCD a block lands on,
// and the index-ordered final sum is bitwise reproducible.
//
// Two-level ticket: workgroup b counts in group b % G (G = kTicketGroups counters, each on
// its own 256-byte line); the last arrival of each group takes the top-level ticket, and the
// last of those reduces. One same-address counter serialised 2048 near-simultaneous atomics
// at the end of every launch (~14 us at N = 1e8, profiles/r1/overhead_n_sweep.jsonl).
#pragma once

#include <hip/hip_runtime.h>

#include "miint/kernels.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {

constexpr int kFinalBatch = 16;  // partial loads in flight per thread

// Thread t sums partials t, t + BLOCK, t + 2 BLOCK, ... in increasing order. The loads of a
// batch are all issued before the first add (a plain loop waited for every load).
template <int BLOCK, bool AGENT_SCOPE>
__device__ __forceinline__ double ordered_partials(const double* partials, int n) {
  double v = 0.0;
  for (int base = 0; base < n; base += kFinalBatch * BLOCK) {
    double r[kFinalBatch];
#pragma unroll
    for (int k = 0; k < kFinalBatch; ++k) {
      const int i = base + k * BLOCK + static_cast<int>(threadIdx.x);
      if constexpr (AGENT_SCOPE)
        r[k] = i < n ? __hip_atomic_load(&partials[i], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT)
                     : 0.0;
      else
        r[k] = i < n ? partials[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kFinalBatch; ++k) v += r[k];
  }
  return v;
}

// Publish this workgroup's partial s (thread 0's value) as partials[bid] and take the
// ticket. Returns true, uniformly across the workgroup, in the last of `nblocks`
// workgroups, which may then read every partial with ordered_partials<BLOCK, true>.
// `flag` is a __shared__ int of the caller.
__device__ __forceinline__ bool publish_and_ticket(double s, double* partials, unsigned* ticket,
                                                   unsigned bid, unsigned nblocks, int* flag) {
  const unsigned G = nblocks < kTicketGroups ? nblocks : kTicketGroups;
  if (threadIdx.x == 0) {
    __hip_atomic_store(&partials[bid], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned g = bid % G;
    const unsigned members = (nblocks - g + G - 1) / G;
    const unsigned prev = __hip_atomic_fetch_add(ticket + g * kTicketStride, 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = 0;
    if (prev == members - 1) {
      const unsigned top = __hip_atomic_fetch_add(ticket + kTicketGroups * kTicketStride, 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (top == G - 1);
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return true;
}

// Re-arm the ticket (last workgroup only: every group has arrived, nobody else touches it).
__device__ __forceinline__ void rearm_ticket(unsigned* ticket, unsigned nblocks) {
  const unsigned G = nblocks < kTicketGroups ? nblocks : kTicketGroups;
  if (threadIdx.x < G)
    __hip_atomic_store(ticket + threadIdx.x * kTicketStride, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0)
    __hip_atomic_store(ticket + kTicketGroups * kTicketStride, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace miint
