// Wave64 reductions and scans built on gfx9-family DPP (data-parallel primitives).
//
// This is the MI355X-native replacement for the reference's reductions, which are:
//   * per-thread serial sums + host serial sum of 64 partials (cintegrate.cu:66-71, 133-138)
//   * a hand-rolled MPI gather to rank 0 (riemann.cpp:76, 82-85)
// Here the reduction happens in registers: fp64 values move between lanes with
// v_mov_b32_dpp (two per double: DPP is a 32-bit VOP1/VOP2 modifier on gfx950), fp32
// values fold directly into v_add_f32_dpp. Inside a row (16 lanes) we use
// quad_perm / row_half_mirror / row_mirror, across rows the gfx9-only row_bcast:15 and
// row_bcast:31 controls. No LDS traffic until the cross-wave step.
//
// Determinism: every function here performs a fixed sequence of additions independent of
// timing, so repeated launches are bitwise identical (tests/test_gpu_kernels.py checks it).
#pragma once

#include <hip/hip_runtime.h>

namespace miint {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// DPP control words (gfx9 encoding).
enum : int {
  kDppQuadXor1 = 0xB1,      // quad_perm:[1,0,3,2]
  kDppQuadXor2 = 0x4E,      // quad_perm:[2,3,0,1]
  kDppRowShr1 = 0x111,
  kDppRowShr2 = 0x112,
  kDppRowShr4 = 0x114,
  kDppRowShr8 = 0x118,
  kDppRowMirror = 0x140,    // lane i <- lane 15-i within a row
  kDppRowHalfMirror = 0x141,// lane i <- lane 7-i within a half-row
  kDppRowBcast15 = 0x142,   // lane 15 of row r -> every lane of row r+1
  kDppRowBcast31 = 0x143,   // lane 31 -> every lane of rows 2 and 3
};

// Move `v` across lanes with DPP; lanes whose row is masked off (or whose source is out
// of range, bound_ctrl=0) receive `old`.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ double dpp(double v, double old = 0.0) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, BANK_MASK, false);
}
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ float dpp(float v, float old = 0.0f) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, BANK_MASK, false);
}

// A lane permutation inside each row (quad_perm, row mirrors: every lane has a source lane,
// every row is written): no `old` value is read, so none is materialised — dpp<>()'s old = 0
// costs a v_mov_b32 per 32-bit half at every step (2 per fp64 step).
template <int CTRL>
__device__ __forceinline__ double dpp_perm(double v) {
  const long long bits = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(bits), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(bits >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}
template <int CTRL>
__device__ __forceinline__ float dpp_perm(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over each row of 16 lanes (every lane of the row holds it) in 4 steps.
template <typename T>
__device__ __forceinline__ T row_sum(T v) {
  v += dpp_perm<kDppQuadXor1>(v);
  v += dpp_perm<kDppQuadXor2>(v);
  v += dpp_perm<kDppRowHalfMirror>(v);
  v += dpp_perm<kDppRowMirror>(v);          // every lane: its row's sum
  return v;
}

// Full-wave sum. Returns the total in lane 63 (other lanes hold partial sums); use
// wave_broadcast_last() when every lane needs it.
template <typename T>
__device__ __forceinline__ T wave_sum_to_last(T v) {
  v = row_sum(v);
  v += dpp<kDppRowBcast15, 0xA>(v);         // rows 1,3 += rows 0,2
  v += dpp<kDppRowBcast31, 0xC>(v);         // rows 2,3 += (row0+row1)
  return v;                                 // lane 63 = total
}

// Sum of lanes 0 .. N-1 (N <= 16; every other lane holds 0) in lane 0: the steps of
// wave_sum_to_last that combine non-zero values — the rest only add zeros — so the value is
// bitwise wave_sum_to_last's lane 63 (up to the sign of an exact zero). The cross-wave step
// of a block sum (4 wave totals at 256 threads, 16 at 1024): 2 or 4 DPP steps on the
// critical path after the barrier instead of 6.
template <typename T>
__device__ __forceinline__ T lanes_sum_small(T v, int n) {
  v += dpp_perm<kDppQuadXor1>(v);
  v += dpp_perm<kDppQuadXor2>(v);
  if (n > 4) {
    v += dpp_perm<kDppRowHalfMirror>(v);
    v += dpp_perm<kDppRowMirror>(v);
  }
  return v;  // lanes 0..3 (n <= 4) or 0..15: the sum
}
__device__ __forceinline__ double wave_broadcast_first(double v) {
  const long long bits = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(bits));
  const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(bits >> 32));
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}
__device__ __forceinline__ float wave_broadcast_first(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

__device__ __forceinline__ double wave_broadcast_last(double v) {
  const long long bits = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(bits), 63);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), 63);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}
__device__ __forceinline__ float wave_broadcast_last(float v) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  return wave_broadcast_last(wave_sum_to_last(v));
}

// Inclusive wave scan (Hillis-Steele within rows, then row_bcast carries).
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
  v += dpp<kDppRowShr1>(v);
  v += dpp<kDppRowShr2>(v);
  v += dpp<kDppRowShr4>(v);
  v += dpp<kDppRowShr8>(v);
  v += dpp<kDppRowBcast15, 0xA>(v);
  v += dpp<kDppRowBcast31, 0xC>(v);
  return v;
}

// Block-wide sum: DPP inside each wave, then one value per wave through LDS, then DPP
// again in wave 0. `lds` must hold at least NWAVES elements. Result valid in thread 0
// (and returned to every thread of wave 0's lane 63 path via broadcast).
template <int BLOCK, typename T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  static_assert(BLOCK % kWave == 0 && BLOCK <= 1024, "block must be whole waves");
  constexpr int kNW = BLOCK / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  v = wave_sum_to_last(v);
  if constexpr (kNW == 1) {
    return wave_broadcast_last(v);
  } else {
    if (lane == kWave - 1) lds[wid] = v;
    __syncthreads();
    T r = T(0);
    if (wid == 0) {
      r = lane < kNW ? lds[lane] : T(0);
      r = kNW <= 16 ? wave_broadcast_first(lanes_sum_small(r, kNW)) : wave_sum(r);
    }
    return r;  // meaningful in wave 0
  }
}

// block_sum for a block size chosen at launch (blockDim.x: whole waves, <= 1024; `lds` holds
// at least blockDim.x / kWave elements). For blockDim.x == BLOCK it performs exactly
// block_sum<BLOCK>'s additions, so results are bitwise the same.
template <typename T>
__device__ __forceinline__ T block_sum_dyn(T v, T* lds) {
  const int nw = static_cast<int>(blockDim.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  v = wave_sum_to_last(v);
  if (nw == 1) return wave_broadcast_last(v);
  if (lane == kWave - 1) lds[wid] = v;
  __syncthreads();
  T r = T(0);
  if (wid == 0) {
    r = lane < nw ? lds[lane] : T(0);
    r = wave_broadcast_first(lanes_sum_small(r, nw));  // nw <= 16
  }
  return r;  // meaningful in wave 0
}

// block_sum_dyn of C independent values at once (`lds` holds C * 16 elements): per value
// exactly block_sum_dyn's additions, so each out[c] is bitwise block_sum_dyn(v[c]). The C
// DPP chains interleave (each hides the others' DPP wait states and latency) and the block
// pays one barrier for all C — the multi-step kernel's per-step sum at one wave per SIMD,
// where a single chain and a barrier every step have no other wave to issue from.
template <int C, typename T>
__device__ __forceinline__ void block_sums_dyn(T (&v)[C], T* lds, T (&out)[C]) {
  constexpr int kSlots = 16;  // wave totals per value (<= 1024 threads)
  const int nw = static_cast<int>(blockDim.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = wave_sum_to_last(v[c]);
  if (nw == 1) {
#pragma unroll
    for (int c = 0; c < C; ++c) out[c] = wave_broadcast_last(v[c]);
    return;
  }
  if (lane == kWave - 1) {
#pragma unroll
    for (int c = 0; c < C; ++c) lds[c * kSlots + wid] = v[c];
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) out[c] = T(0);
  if (wid == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const T r = lane < nw ? lds[c * kSlots + lane] : T(0);
      out[c] = wave_broadcast_first(lanes_sum_small(r, nw));
    }
  }
}

// Block-wide inclusive scan; also returns the block total through *total.
template <int BLOCK, typename T>
__device__ __forceinline__ T block_inclusive_scan(T v, T* lds, T* total) {
  constexpr int kNW = BLOCK / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  v = wave_inclusive_scan(v);
  if (lane == kWave - 1) lds[wid] = v;
  __syncthreads();
  if (wid == 0) {
    T w = lane < kNW ? lds[lane] : T(0);
    w = wave_inclusive_scan(w);
    if (lane < kNW) lds[lane] = w;  // inclusive prefix over waves
  }
  __syncthreads();
  if (wid > 0) v += lds[wid - 1];
  *total = lds[kNW - 1];
  return v;
}

}  // namespace miint
