// Fused two-phase train-profile scan for gfx950: velocity samples -> running integral
// ("distance", 4main.c phase 1) -> running integral of that ("sum of sums", phase 2),
// written in ONE write-only pass over HBM.
//
// Reference (4main.c:76-221): fill 144 MB, local serial scan, gather all
// slices to rank 0, serial carry loop on rank 0, 144 MB broadcast; then the same again for
// phase 2. Its inputs are never data: every velocity sample is interp(profile, i*dt).
// That makes a reduce-then-scan free of input reads:
//
//   K1 ts_tile_sums   per 4096-sample tile t: S1 = sum_i v_i and S2 = sum_i (n_t - i) v_i
//                     (the sum of the tile's local inclusive prefix sums) — compute only
//   K2 ts_tile_prefix one workgroup: P1(t) = sum_{u<t} S1(u),
//                     Q(t) = sum_{u<t} [n_u P1(u) + S2(u)]   (DPP/LDS block scans), and the
//                     rank totals T1 = P1(end), T2 = Q(end)
//   (multi-GPU)       allgather (T1, T2, count) per rank -> rank carries C1, C2 (K3)
//   K4 ts_write       per tile: recompute v, vel = C1 + P1(t) + local scan(v),
//                     pos = C2 + 4096 t C1 + Q(t) + local scan(vel); both transposed through
//                     LDS and stored with coalesced 16-byte stores
//
// HBM traffic: 2 x 8 bytes per sample, written once (vel, pos); nothing is read back.
// The 4main --parity fill windows (rank-private fills, 4main.c:76-86) are honoured: samples
// outside [win_lo, win_hi) are zero.
#include <hip/hip_runtime.h>

#include "miint/common.hpp"
#include "miint/trainscan.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {
namespace {

constexpr int kB = 256;
constexpr int kItems = 16;
constexpr int kTile = kB * kItems;  // 4096 samples
constexpr int kMaxTable = 2048;
constexpr int kSpan = 64;  // table entries staged per tile (LDS)
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const double lds_f64;

struct Sampler {
  const double* tab;  // LDS copy of table entries [s0, s0 + count), or the global table
  bool staged;        // tab points into LDS
  int s0, nseg;
  double dt;
  uint64_t i0, n, win_lo, win_hi;
  __device__ __forceinline__ double operator()(uint64_t g) const {  // g: slice-local index
    const uint64_t i = i0 + g;
    if (g >= n || i < win_lo || i >= win_hi) return 0.0;
    const double t = dt * static_cast<double>(i);
    int s = static_cast<int>(t);
    s = s < 0 ? 0 : (s >= nseg ? nseg - 1 : s);
    const double v0 = tab[s - s0];
    return fma(tab[s + 1 - s0] - v0, t - static_cast<double>(s), v0);
  }
  // The kItems consecutive samples of this thread, starting at slice-local index g.
  // Hot form (tile fully inside the slice and the fill window): 64-bit index math once per
  // thread, then per sample t = fma(k, dt, t_first), a 32-bit segment index and two
  // broadcast LDS reads — identical to operator() up to one rounding of t.
  // The hot form only runs on staged tiles and reads through an LDS-typed pointer: through
  // the generic pointer the compiler emits flat_load_dwordx4 pairs (8-byte aligned 16-byte
  // LDS reads: SQ_LDS_UNALIGNED_STALL 3.8e6 per pass) instead of ds_read2_b64.
  __device__ __forceinline__ void items(uint64_t g, bool plain, double (&v)[kItems]) const {
    if (!plain) {
#pragma unroll
      for (int k = 0; k < kItems; ++k) v[k] = (*this)(g + k);
      return;
    }
    lds_f64* lt = (lds_f64*)tab;
    const double tb = dt * static_cast<double>(i0 + g);
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const double t = fma(static_cast<double>(k), dt, tb);
      int s = static_cast<int>(t);
      s = s >= nseg ? nseg - 1 : s;
      const double v0 = lt[s - s0];
      v[k] = fma(lt[s + 1 - s0] - v0, t - static_cast<double>(s), v0);
    }
  }
  // Block-uniform: can every sample of tile [t0, t0 + kTile) take the hot form?
  __device__ __forceinline__ bool plain_tile(uint64_t t0) const {
    return staged && t0 + kTile <= n && i0 + t0 >= win_lo && i0 + t0 + kTile <= win_hi;
  }
};

__device__ __forceinline__ int seg_of(double t, int nseg) {
  int s = static_cast<int>(t);
  return s < 0 ? 0 : (s >= nseg ? nseg - 1 : s);
}

// Stage only the table entries this tile's samples touch: a 4096-sample tile at 1e4
// samples/s spans 0.41 s, i.e. 2-3 entries instead of the whole 14.4 KB table per
// workgroup (the full re-staging cost 63 MB of L2 reads per pass).
__device__ __forceinline__ Sampler make_sampler(const TrainScanKernelParams& p, double* tab) {
  const int nseg = p.table_n - 1;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile;
  const uint64_t last = (t0 + kTile < p.n ? t0 + kTile : p.n) - 1;
  const int s0 = seg_of(p.dt * static_cast<double>(p.i0 + t0), nseg);
  const int s1 = seg_of(p.dt * static_cast<double>(p.i0 + last), nseg) + 1;
  if (s1 - s0 + 1 > kSpan)  // coarse sampling: read the (L2-resident) table directly
    return {p.table, false, 0, nseg, p.dt, p.i0, p.n, p.win_lo, p.win_hi};
  for (int k = threadIdx.x; k <= s1 - s0; k += kB) tab[k] = p.table[s0 + k];
  __syncthreads();
  return {tab, true, s0, nseg, p.dt, p.i0, p.n, p.win_lo, p.win_hi};
}

// ---------------------------------------------------------------------------- K1
__global__ __launch_bounds__(kB) void ts_tile_sums(TrainScanKernelParams p, f64x2* sums) {
  __shared__ double tab[kSpan];
  __shared__ double red1[kB / kWave], red2[kB / kWave];
  const Sampler f = make_sampler(p, tab);
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile;
  const uint64_t nt = p.n - t0 < kTile ? p.n - t0 : kTile;
  double v[kItems];
  f.items(t0 + threadIdx.x * kItems, f.plain_tile(t0), v);
  const double w0 = static_cast<double>(static_cast<int64_t>(nt) - threadIdx.x * kItems);
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    s1 += v[k];
    s2 = fma(w0 - k, v[k], s2);  // sample i is counted n_t - i times in the tile's prefixes
  }
  s1 = block_sum<kB>(s1, red1);
  s2 = block_sum<kB>(s2, red2);
  if (threadIdx.x == 0) sums[blockIdx.x] = f64x2{s1, s2};
}

// ---------------------------------------------------------------------------- K2
constexpr int kPB = 1024;
__global__ __launch_bounds__(kPB) void ts_tile_prefix(const f64x2* sums, uint32_t ntiles,
                                                      uint64_t n, f64x2* prefix, double* totals) {
  __shared__ double red[kPB / kWave];
  double c1 = 0.0, c2 = 0.0;  // running carries over chunks (uniform)
  for (uint32_t base = 0; base < ntiles; base += kPB) {
    const uint32_t t = base + threadIdx.x;
    const f64x2 s = t < ntiles ? sums[t] : f64x2{0.0, 0.0};
    const uint64_t t0 = static_cast<uint64_t>(t) * kTile;
    const double nt = t < ntiles ? static_cast<double>(n - t0 < kTile ? n - t0 : kTile) : 0.0;
    double tot1;
    const double incl1 = block_inclusive_scan<kPB>(s.x, red, &tot1);
    const double p1 = c1 + (incl1 - s.x);  // exclusive prefix of S1
    __syncthreads();
    const double q = fma(nt, p1, s.y);
    double tot2;
    const double incl2 = block_inclusive_scan<kPB>(q, red, &tot2);
    if (t < ntiles) prefix[t] = f64x2{p1, c2 + (incl2 - q)};
    c1 += tot1;
    c2 += tot2;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    totals[0] = c1;  // T1: slice sum of v
    totals[1] = c2;  // T2: slice sum of the local running integral
  }
}

// ---------------------------------------------------------------------------- K3
// gathered: world x {T1, T2, count}. carries = {C1, C2} for `rank` (fixed order everywhere).
__global__ void ts_rank_carry(const double* gathered, int rank, double* carries) {
  double c1 = 0.0, c2 = 0.0;
  for (int q = 0; q < rank; ++q) {
    const double t1 = gathered[3 * q], t2 = gathered[3 * q + 1], cnt = gathered[3 * q + 2];
    c2 += fma(cnt, c1, t2);  // rank q's position total = count_q * C1(q) + T2(q)
    c1 += t1;
  }
  carries[0] = c1;
  carries[1] = c2;
}

// ---------------------------------------------------------------------------- K4
// 16-byte chunk c of the tile lives at LDS chunk c ^ ((c >> 3) & 15): conflict-free for
// both sides of the transpose (MI355X_MICROARCH.md §LDS) — the ds_write_b128 of thread t
// (chunks 8t..8t+7, 8 contiguous lanes per group, banks (a/4) mod 32) and the ds_read_b128
// of chunk k*256 + t (4 non-contiguous 16-lane groups, banks (a/4) mod 64). A +16 B per
// 128 B padding was conflict-free only for the writes (1.1e6 conflict cycles per pass).
__device__ __forceinline__ int swz(int c) { return c ^ ((c >> 3) & 15); }

__device__ __forceinline__ void store_tile(double* buf, const double (&v)[kItems], double* out,
                                           uint64_t t0, uint64_t n) {
  // blocked (thread-contiguous) -> LDS -> striped 16-byte stores
#pragma unroll
  for (int k = 0; k < kItems; k += 2) {
    const int c = swz((threadIdx.x * kItems + k) >> 1);
    *reinterpret_cast<f64x2*>(&buf[2 * c]) = f64x2{v[k], v[k + 1]};
  }
  __syncthreads();
  const bool full = t0 + kTile <= n;
#pragma unroll
  for (int k = 0; k < kItems / 2; ++k) {
    const int e = 2 * (k * kB + threadIdx.x);  // element pair index within the tile
    const f64x2 w = *reinterpret_cast<const f64x2*>(&buf[2 * swz(e >> 1)]);
    if (full) {
      *reinterpret_cast<f64x2*>(&out[t0 + e]) = w;
    } else {
      if (t0 + e < n) out[t0 + e] = w.x;
      if (t0 + e + 1 < n) out[t0 + e + 1] = w.y;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kB) void ts_write(TrainScanKernelParams p, const f64x2* prefix,
                                               const double* carries, double* vel, double* pos) {
  __shared__ double tab[kSpan];
  __shared__ double red[kB / kWave];
  __shared__ __attribute__((aligned(16))) double buf[kTile];
  const Sampler f = make_sampler(p, tab);
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile;
  const f64x2 pr = prefix[blockIdx.x];
  const double c1 = carries ? carries[0] : 0.0;
  const double c2 = carries ? carries[1] : 0.0;
  double v[kItems];
  f.items(t0 + threadIdx.x * kItems, f.plain_tile(t0), v);
  double run = 0.0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    run += v[k];
    v[k] = run;  // thread-local inclusive scan of the samples
  }
  double tot;
  const double ex1 = block_inclusive_scan<kB>(run, red, &tot) - run;
  const double base1 = (c1 + pr.x) + ex1;
#pragma unroll
  for (int k = 0; k < kItems; ++k) v[k] += base1;  // velocity integral ("distance")
  if (vel) store_tile(buf, v, vel, t0, p.n);
  __syncthreads();
  run = 0.0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    run += v[k];
    v[k] = run;
  }
  const double ex2 = block_inclusive_scan<kB>(run, red, &tot) - run;
  const double base2 = (c2 + fma(static_cast<double>(t0), c1, pr.y)) + ex2;
#pragma unroll
  for (int k = 0; k < kItems; ++k) v[k] += base2;  // running integral of the above
  if (pos) store_tile(buf, v, pos, t0, p.n);
}

}  // namespace

size_t trainscan_workspace_bytes(uint64_t n) {
  const uint64_t nt = (n + kTile - 1) / kTile;
  return 2 * nt * sizeof(f64x2) + 64;
}

void launch_trainscan_local(const TrainScanKernelParams& p, void* ws, double* totals,
                            hipStream_t s) {
  MIINT_CHECK(p.n >= 1, "empty slice");
  MIINT_CHECK(p.table_n >= 2 && p.table_n <= kMaxTable, "table size must be in [2, 2048]");
  const uint64_t nt = (p.n + kTile - 1) / kTile;
  MIINT_CHECK(nt < (1u << 31), "slice too large");
  f64x2* sums = static_cast<f64x2*>(ws);
  f64x2* prefix = sums + nt;
  ts_tile_sums<<<static_cast<unsigned>(nt), kB, 0, s>>>(p, sums);
  MIINT_HIP(hipGetLastError());
  ts_tile_prefix<<<1, kPB, 0, s>>>(sums, static_cast<uint32_t>(nt), p.n, prefix, totals);
  MIINT_HIP(hipGetLastError());
}

void launch_trainscan_rank_carry(const double* gathered, int rank, double* carries,
                                 hipStream_t s) {
  ts_rank_carry<<<1, 1, 0, s>>>(gathered, rank, carries);
  MIINT_HIP(hipGetLastError());
}

void launch_trainscan_write(const TrainScanKernelParams& p, const void* ws, const double* carries,
                            double* vel, double* pos, hipStream_t s) {
  MIINT_CHECK((reinterpret_cast<uintptr_t>(vel) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(pos) & 15) == 0,
              "trainscan outputs need 16-B alignment");
  const uint64_t nt = (p.n + kTile - 1) / kTile;
  const f64x2* prefix = static_cast<const f64x2*>(ws) + nt;
  ts_write<<<static_cast<unsigned>(nt), kB, 0, s>>>(p, prefix, carries, vel, pos);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
