// Cross-workgroup hand-offs inside one launch: write-once slots + last-workgroup ticket.
//
// Write-once slot protocol (used by every in-kernel hand-off: the fused Riemann and 2-D
// field reductions here, the look-back scans in scan.hip and trainscan.hip, the trainscan
// block-prefix ticket): a slot holds kUnset — a NaN bit pattern no arithmetic produces —
// until its producer stores the value with ONE relaxed agent-scope atomic store; a consumer
// reads THE SLOT ITSELF with relaxed agent-scope atomic loads until it is no longer kUnset.
// The value is its own flag, so there is no second object whose visibility would have to be
// ordered against it: C++/HIP coherence of a single atomic object is all the protocol needs
// (no release/acquire pair, no reliance on address or control dependencies, nothing a
// compiler may reorder). On gfx950 the relaxed agent-scope forms are sc1 (L1-bypassing,
// write-through) stores and loads, so a consumer never sees a stale line either
// (MI355X_MICROARCH.md "Valid forms"); the producer's s_waitcnt vmcnt(0) before its ticket
// only makes the slot usually visible by the time the ticket is counted (no spin). Slots
// are re-armed to kUnset by their single consumer once read, or by the launcher's memset.
// Every wait is bounded: a slot still unset after kSlotSpinLimit polls reads as NaN (and
// raises the caller's timeout word), which poisons the result instead of hanging the GPU.
//
// Last-workgroup ticket (fused reductions): every workgroup publishes its partial into its
// slot, then takes a ticket with an agent-scope atomic; the workgroup that draws the last
// ticket reduces all slots in index order (bitwise reproducible, placement-independent —
// cdna_hip_programming.md §6 G16) and re-arms them.
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

// ---------------------------------------------------------------- write-once slots
// both 32-bit halves kUnsetSlotWord (kernels.hpp), so hipMemsetD32 fills slots; a quiet NaN
// with a payload no arithmetic produces
constexpr unsigned long long kUnsetBits =
    (static_cast<unsigned long long>(kUnsetSlotWord) << 32) | kUnsetSlotWord;
constexpr unsigned kSlotSpinLimit = 1u << 26;

__device__ __forceinline__ bool slot_unset(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v)) == kUnsetBits;
}
__device__ __forceinline__ double slot_unset_value() {
  return __longlong_as_double(static_cast<long long>(kUnsetBits));
}
__device__ __forceinline__ double slot_load(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void slot_store(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait until the slot is set; NaN (and *timeout = 1, if given) after kSlotSpinLimit polls.
__device__ __forceinline__ double slot_wait(const double* p, double first,
                                            unsigned* timeout = nullptr) {
  double v = first;
  unsigned spins = 0;
  while (slot_unset(v)) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kSlotSpinLimit) {
      if (timeout) __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return __builtin_nan("");
    }
    v = slot_load(p);
  }
  return v;
}

// Thread t sums partials t, t + BLOCK, t + 2 BLOCK, ... in increasing order. The loads of a
// batch are all issued before the first add (a plain loop waited for every load).
// SLOTS = true: the partials are write-once slots of this launch (waited for, see above);
// false: plain loads of partials a previous launch wrote (the kernel boundary orders them),
// or, with SC1, sc1 loads of partials this launch stored write-through before a counted
// arrival the caller has already seen complete (close_batch_in_launch).
// BLOCK = 0: the launch's own block size (blockDim.x), for kernels launched at several sizes.
template <int BLOCK, bool SLOTS, bool SC1 = false>
__device__ __forceinline__ double ordered_partials(const double* partials, int n) {
  const int bs = BLOCK > 0 ? BLOCK : static_cast<int>(blockDim.x);
  double v = 0.0;
  for (int base = 0; base < n; base += kFinalBatch * bs) {
    double r[kFinalBatch];
#pragma unroll
    for (int k = 0; k < kFinalBatch; ++k) {
      const int i = base + k * bs + static_cast<int>(threadIdx.x);
      if constexpr (SLOTS || SC1)
        r[k] = i < n ? slot_load(&partials[i]) : 0.0;
      else
        r[k] = i < n ? partials[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kFinalBatch; ++k) {
      if constexpr (SLOTS) {
        const int i = base + k * bs + static_cast<int>(threadIdx.x);
        if (slot_unset(r[k])) r[k] = slot_wait(&partials[i], r[k]);
      }
      v += r[k];
    }
  }
  return v;
}

// Re-arm slots [0, n) after this thread's ordered_partials<BLOCK, true> read them (each
// thread re-arms exactly the slots it read).
template <int BLOCK>
__device__ __forceinline__ void rearm_slots(double* partials, int n) {
  const int bs = BLOCK > 0 ? BLOCK : static_cast<int>(blockDim.x);
  for (int i = static_cast<int>(threadIdx.x); i < n; i += bs)
    slot_store(&partials[i], slot_unset_value());
}

// Publish this workgroup's partial s (thread 0's value) into slot partials[bid] and take the
// ticket. Returns true, uniformly across the workgroup, in the last of `nblocks`
// workgroups, which may then read every slot with ordered_partials<BLOCK, true> (and must
// re-arm them with rearm_slots). `flag` is a __shared__ int of the caller.
__device__ __forceinline__ bool publish_and_ticket(double s, double* partials, unsigned* ticket,
                                                   unsigned bid, unsigned nblocks, int* flag) {
  const unsigned G = nblocks < kTicketGroups ? nblocks : kTicketGroups;
  if (threadIdx.x == 0) {
    slot_store(&partials[bid], s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // latency only: see the header
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
  return *flag != 0;  // the slots are read as atomics: no acquire fence needed
}

// In-launch close of a multi-step batch (RiemannConfig::close, "launch"): the persistent
// launch's own workgroups turn its `steps` rows of `nb` step partials into the step values
// out[s] = scale * (row s summed exactly as multistep_close_kernel sums it) — no closing
// kernel, no kernel boundary after the launch.
//  * Every workgroup's thread 0 stored ALL of its step partials write-through (slot_store,
//    sc1), then waits for them (s_waitcnt vmcnt(0)) and counts the workgroup in shard
//    b % S (S = min(kTicketGroups, nb) counters, each on its own 256-byte line: one counter
//    serialised ~12 ns per arrival, MI355X_MICROARCH.md "fanin").
//  * The last arrival of shard c becomes closer c: its wave 0 polls every shard (lane l
//    loads shard l, sc1, s_sleep between polls, bounded) until all nb workgroups have
//    arrived, then the workgroup barrier releases the closer's other waves, and all of them
//    read the rows with sc1 loads: the first row of the sc1 hand-off table in
//    MI355X_MICROARCH.md "Valid forms" (one lane per storing workgroup for all its stores,
//    agent-scope adds, an sc1 poll of every shard, a barrier before the other waves load).
//  * Closer c closes steps c, c + S, ...: ordered_partials + block_sum_dyn at the launch's
//    block size, the closing kernel's arithmetic, so the values are bitwise the same.
//  * The closer whose count on the done line (after the shards) is last re-arms every
//    counter to zero for the next launch; no other workgroup reads them after its poll.
// Spinning is safe where the close kernel was not needed: only the last arrival of each
// shard waits, for workgroups already past their last step (at most S closers hold slots
// while every other workgroup has exited). A poll that hits kSlotSpinLimit writes NaN
// results instead of hanging the GPU.
// `ticket` holds kTicketWords words, zero before the first launch.
__device__ __forceinline__ void close_batch_in_launch(const double* partials, unsigned nb,
                                                      int steps, unsigned* ticket, double scale,
                                                      double* out, double* red, int* role) {
  const unsigned S = nb < static_cast<unsigned>(kTicketGroups) ? nb : kTicketGroups;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's sc1 partials landed
    const unsigned g = blockIdx.x % S;
    const unsigned members = (nb - g + S - 1) / S;
    const unsigned prev = __hip_atomic_fetch_add(ticket + g * kTicketStride, 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *role = prev == members - 1 ? static_cast<int>(g) : -1;
  }
  __syncthreads();
  const int c = *role;
  if (c < 0) return;
  __shared__ int timed_out;
  if (threadIdx.x < kWave) {
    const unsigned lane = threadIdx.x;
    const unsigned want = lane < S ? (nb - lane + S - 1) / S : 0u;
    int late = 0;
    for (unsigned spins = 0;; ++spins) {
      const unsigned got =
          lane < S ? __hip_atomic_load(ticket + lane * kTicketStride, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
      if (__all(got >= want)) break;
      if (spins > kSlotSpinLimit) {
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) timed_out = late;
  }
  __syncthreads();
  const bool bad = timed_out != 0;
  for (int s = c; s < steps; s += static_cast<int>(S)) {
    const double t = ordered_partials<0, false, true>(partials + static_cast<size_t>(s) * nb,
                                                      static_cast<int>(nb));
    const double tot = block_sum_dyn(t, red);
    if (threadIdx.x == 0) out[s] = bad ? __builtin_nan("") : tot * scale;
    __syncthreads();  // red is reused by the next step
  }
  if (threadIdx.x == 0) {
    const unsigned d = __hip_atomic_fetch_add(ticket + kTicketGroups * kTicketStride, 1u,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == S - 1) {  // every closer is past its poll: re-arm for the next launch
      for (unsigned g = 0; g < S; ++g)
        __hip_atomic_store(ticket + g * kTicketStride, 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ticket + kTicketGroups * kTicketStride, 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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
