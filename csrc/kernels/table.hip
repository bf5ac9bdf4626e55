// Table kernels for gfx950: HBM-bound array sum, interpolated-profile fill, and the 2-D
// bilinear field integral.
//
// Reference counterparts:
//   cuda_test pass 1  cintegrate.cu:88-92  d_InterpProfile[i] = faccel(i*dt) — 3 global
//                     loads/sample, per-thread contiguous chunks (uncoalesced stores)
//   cuda_test pass 2  cintegrate.cu:94-96  serial re-read of the 144 MB array per thread
//   4main fill        4main.c:82-86        same fill on the host
// Here: the fill gives each workgroup one contiguous chunk and stages only the table window
// that chunk touches in LDS; the sum walks the array grid-stride; both move 16 bytes per lane
// per access (global_store_dwordx4 / global_load_dwordx4) over 64-bit indices.
// The 2-D config (BASELINE.json #5) has no reference counterpart: it integrates a
// ny x nx fp64 field with bilinear interpolation, each workgroup staging the table
// footprint of its 256-column block of sample rows in LDS (2-D LDS tiling) and streaming
// down the rows.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "miint/common.hpp"
#include "miint/handoff.hpp"
#include "miint/kernels.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {
namespace {

constexpr int kB = 256;
typedef double f64x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------- sum_array
// Four 16-byte loads in flight per lane per iteration; fixed assignment of elements to
// lanes -> deterministic.
__global__ __launch_bounds__(kB) void sum_array_kernel(const double* __restrict__ x, uint64_t n,
                                                       double* partials) {
  __shared__ double red[kB / kWave];
  const uint64_t nv = n / 2;  // number of double2 vectors
  const f64x2* xv = reinterpret_cast<const f64x2*>(x);
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * kB;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * kB + threadIdx.x;
  f64x2 a0 = {0.0, 0.0}, a1 = a0, a2 = a0, a3 = a0;
  for (; i + 3 * lanes < nv; i += 4 * lanes) {
    const f64x2 v0 = xv[i], v1 = xv[i + lanes], v2 = xv[i + 2 * lanes], v3 = xv[i + 3 * lanes];
    a0 += v0; a1 += v1; a2 += v2; a3 += v3;
  }
  for (; i < nv; i += lanes) a0 += xv[i];
  double acc = (a0.x + a0.y) + (a1.x + a1.y) + ((a2.x + a2.y) + (a3.x + a3.y));
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kB + threadIdx.x;
  if ((n & 1) && gid == 0) acc += x[n - 1];
  const double s = block_sum<kB>(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// ---------------------------------------------------------------------------- interp fill
constexpr int kMaxTable = 2048;
constexpr uint64_t kFillBlocks = 2048;

// Clamped segment of time t (in table steps): clamped in fp64 before the conversion, so a t
// beyond the int range is the last segment, not an undefined conversion.
__device__ __forceinline__ int seg_of(double t, int nseg) {
  return t >= static_cast<double>(nseg) ? nseg - 1 : (t < 1.0 ? 0 : static_cast<int>(t));
}

// set_lds_poison: NaN in every LDS word a window does not stage (validation only); the 2-D
// stream kernel gets it as a template instantiation instead (no branch in the hot kernel)
__constant__ int g_lds_poison;
std::atomic<bool> g_table2d_poison{false};

__device__ __forceinline__ double interp_lds(const double* tab, int nseg, double t) {
  const int i = seg_of(t, nseg);
  const double v0 = tab[i];
  return fma(tab[i + 1] - v0, t - static_cast<double>(i), v0);
}

// Each workgroup owns one contiguous chunk of the output (C double2 vectors, walked 256 at a
// time: every pass is one coalesced 4 KB store) and stages only the table entries its chunk
// can touch, [k0, k1 + 1]: the clamped segment index is monotonic in the sample index, so
// the chunk's first and last samples bound it. At the reference's 10 000 samples/s a
// 2048-workgroup fill of 18e6 samples touches 2-3 entries per workgroup; the grid-stride form
// this replaced staged the whole 1801-entry table in each of 8192 workgroups (118 MB of L2
// reads beside 144 MB of stores): 28.2-29.4 -> 23.4-23.7 us, 5.0 -> 6.1 TB/s, measured
// alternately in one process per build (profiles/r2/interp_fill_ab.jsonl; tools/fill_ab.sh).
// One store per lane per pass: unrolling by 4, or 1024 / 4096 workgroups, measured 24.0 us.
__global__ __launch_bounds__(kB) void interp_fill_kernel(const double* __restrict__ table,
                                                         int table_n, double dt, uint64_t i0,
                                                         uint64_t n, uint64_t chunk,
                                                         double* __restrict__ y) {
  __shared__ double tab[kMaxTable];
  const int nseg = table_n - 1;
  const uint64_t nv = n / 2;
  const uint64_t vb = static_cast<uint64_t>(blockIdx.x) * chunk;
  const uint64_t ve = vb + chunk < nv ? vb + chunk : nv;
  auto seg = [&](uint64_t i) { return seg_of(dt * static_cast<double>(i), nseg); };
  if (vb < ve) {
    const int ka = seg(i0 + 2 * vb), kb = seg(i0 + 2 * ve - 1);
    const int k0 = ka < kb ? ka : kb, k1 = ka < kb ? kb : ka;
    if (g_lds_poison) {
      for (int k = static_cast<int>(threadIdx.x); k < kMaxTable; k += kB) tab[k] = __builtin_nan("");
      __syncthreads();
    }
    for (int k = k0 + static_cast<int>(threadIdx.x); k <= k1 + 1; k += kB) tab[k - k0] = table[k];
    __syncthreads();
    auto at = [&](uint64_t i) {  // interp_lds on the staged window (tab[j] = table[k0 + j])
      const double t = dt * static_cast<double>(i);
      const int k = seg(i);
      const double v0 = tab[k - k0];
      return fma(tab[k - k0 + 1] - v0, t - static_cast<double>(k), v0);
    };
    f64x2* yv = reinterpret_cast<f64x2*>(y);
#pragma unroll 1
    for (uint64_t v = vb + threadIdx.x; v < ve; v += kB) {
      const uint64_t i = i0 + 2 * v;
      yv[v] = f64x2{at(i), at(i + 1)};
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)  // the odd last sample, from global
    y[n - 1] = interp_lds(table, nseg, dt * static_cast<double>(i0 + n - 1));
}

// ---------------------------------------------------------------------------- outer product
__global__ __launch_bounds__(kB) void outer_product_kernel(const double* __restrict__ v, int n,
                                                           double* __restrict__ t) {
  const int j = blockIdx.x * kB + threadIdx.x;
  const int i = blockIdx.y;
  if (j < n) t[static_cast<size_t>(i) * n + j] = v[i] * v[j];
}

// ---------------------------------------------------------------------------- table2d
// Two kernels. Fine sample grids (spacing below ~half a table cell in x, so a workgroup's
// table footprint fits its LDS tile: 4096^2 and up on the 1801^2 field) run the row stream
// below. Coarser grids run this tile kernel, reading the table straight from global memory
// (through L2 and the MALL): workgroup = 16 x 16 threads = one TILE x TILE tile of
// sample points, TILE = 128 (8 x 8 per thread) when the grid gives every CU at least 4
// such tiles, else 64 (4 x 4 per thread).
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Launch modes of both 2-D kernels:
//   kT2Partials  one partial per workgroup (a later finalize sums them)
//   kT2Fused     + last-workgroup hand-off (handoff.hpp): out[0] = the launch's integral
//   kT2Chained   partials, and workgroup 0 first sums the PREVIOUS launch's partials (the
//                other half of a double buffer; the kernel boundary orders them) into
//                *prev_out. In a batch of back-to-back integrations this takes the hand-off
//                tail (slot publish, ticket, one workgroup's ordered read of every slot:
//                2.2-3.4 us, profiles/r2/table2d_tail.jsonl) off the critical path; the
//                batch's last partials are closed by table2d_finalize_kernel.
// Every mode sums the partials with ordered_partials + block_sum in index order, so the
// value is bitwise the same whichever of them produced it.
enum : int { kT2Partials = 0, kT2Fused = 1, kT2Chained = 2 };

struct Table2DChain {
  const double* prev;  // previous launch's partials (kT2Chained; nullptr: nothing to close)
  int prev_n;
  double* prev_out;
};

__device__ __forceinline__ void table2d_close(const double* parts, int n, double* out,
                                              double* red) {
  const double v = ordered_partials<kB, false>(parts, n);
  const double tot = block_sum<kB>(v, red);
  if (threadIdx.x == 0) *out = tot;
  __syncthreads();  // red is reused by the caller's own block_sum
}

__global__ __launch_bounds__(kB) void table2d_finalize_kernel(const double* parts, int n,
                                                              double* out) {
  __shared__ double red[kB / kWave];
  table2d_close(parts, n, out, red);
}

// Per thread: columns c0 + tx + 16 b, rows r0 + ty + 16 a. The column terms (table column,
// fraction) and row terms (row offset, fraction) are computed once per thread — 2 kPer
// index computations instead of kPer^2 (the first form spent 41 VALU per sample) — leaving
// per sample four loads and the bilinear blend. FUSED: the last workgroup reduces all
// partials (handoff.hpp) and writes out[0]; otherwise one partial per workgroup for a
// finalize.
template <int kTile, int MODE>
__global__ __launch_bounds__(kB) void table2d_kernel(Table2DParams p, double* partials,
                                                     unsigned* ticket, double* out,
                                                     Table2DChain chain) {
  constexpr int kPer = kTile / 16;
  __shared__ double red[kB / kWave];
  __shared__ int is_last;
  if constexpr (MODE == kT2Chained) {
    if (chain.prev && blockIdx.x == 0 && blockIdx.y == 0)
      table2d_close(chain.prev, chain.prev_n, chain.prev_out, red);
  }
  const double sx = p.X / p.gx, sy = p.Y / p.gy;          // sample spacing
  const double cx = (p.nx - 1) / p.X, cy = (p.ny - 1) / p.Y;  // table cells per unit
  const int c0 = blockIdx.x * kTile;
  const int r0 = p.row0 + blockIdx.y * kTile;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  size_t col[kPer], row[kPer];
  double fx[kPer], fy[kPer];
#pragma unroll
  for (int b = 0; b < kPer; ++b) {
    const double xx = ((c0 + tx + 16 * b + 0.5) * sx) * cx;
    const int ix = clampi(static_cast<int>(xx), 0, p.nx - 2);
    fx[b] = xx - ix;
    col[b] = ix;
  }
#pragma unroll
  for (int a = 0; a < kPer; ++a) {
    const double yy = ((r0 + ty + 16 * a + 0.5) * sy) * cy;
    const int iy = clampi(static_cast<int>(yy), 0, p.ny - 2);
    fy[a] = yy - iy;
    row[a] = static_cast<size_t>(iy) * p.nx;
  }
  auto sample = [&](int a, int b) {
    const double* t = p.table + (row[a] + col[b]);
    const double v00 = t[0], v01 = t[1], v10 = t[p.nx], v11 = t[p.nx + 1];
    const double top = fma(v01 - v00, fx[b], v00);
    const double bot = fma(v11 - v10, fx[b], v10);
    return fma(bot - top, fy[a], top);
  };
  double acc = 0.0;
  if (c0 + kTile <= p.gx && r0 + kTile <= p.row1) {  // full tile (block-uniform): no checks
#pragma unroll
    for (int a = 0; a < kPer; ++a)
#pragma unroll
      for (int b = 0; b < kPer; ++b) acc += sample(a, b);
  } else {
#pragma unroll
    for (int a = 0; a < kPer; ++a)
#pragma unroll
      for (int b = 0; b < kPer; ++b)
        if (r0 + ty + 16 * a < p.row1 && c0 + tx + 16 * b < p.gx) acc += sample(a, b);
  }
  const double s = block_sum<kB>(acc, red) * (sx * sy);
  const unsigned bid = blockIdx.y * gridDim.x + blockIdx.x;
  if constexpr (MODE != kT2Fused) {
    if (threadIdx.x == 0) partials[bid] = s;
  } else {
    const unsigned nb = gridDim.x * gridDim.y;
    if (!publish_and_ticket(s, partials, ticket, bid, nb, &is_last)) return;
    const double v = ordered_partials<kB, true>(partials, static_cast<int>(nb));
    rearm_slots<kB>(partials, static_cast<int>(nb));
    const double tot = block_sum<kB>(v, red);
    if (threadIdx.x == 0) out[0] = tot;
    rearm_ticket(ticket, nb);
  }
}

// ------------------------------------------------------------------- table2d, row stream
// For fine sample grids (spacing below half a table cell: 4096^2 and up for the 1801^2
// field). Every lane of a wave owns kSCols columns (c0 + lane + 64 b) and all lanes walk the
// SAME rows, so the table row a sample falls in, and its fraction fy, are wave-uniform:
// lane k computes row k's (iy, fy) once, and row k's values come back as SGPRs through
// v_readlane. Per column a lane keeps the x-interpolated lines of the current table row
// pair, Lc (row iy) and D = Ln - Lc (Ln: row iy + 1); each sample is then
//   v = fma(D, fy, Lc),  acc += v                       (2 VALU, fy an SGPR operand)
// — the same value the tile kernel forms (top + fy (bot - top)) — and only when iy moves
// (a scalar compare and branch, once per ~2.3 sample rows at 4096^2) does the lane read
// one ds_read2_b64 for the new line. The LDS tile kernel this replaced read 32 B of LDS and
// spent ~15 VALU per sample; this loop reads ~7 B and ~4 VALU (~11 VALU per sample in all,
// counting staging, column setup and the hand-off at 64 samples per lane).
constexpr int kSCols = 4;                 // columns per lane: a workgroup spans 256 columns
constexpr int kSW = kWave * kSCols / 2;   // LDS footprint width (cells), 128
// LDS footprint height (cells). 30 rows (30 KB tile): 5 workgroups per CU fit the 160 KB of
// LDS where 32 rows fit 4, and the 16-row-per-wave block of a 4096^2 field touches at most
// floor(63 x 0.44) + 3 = 30 table rows. Against 32 (profiles/r4/t2d_variant_ab.jsonl, us per
// integration at 8 step phases): 4096^2 5.34 -> 5.08, 1/2 slice 2.81 -> 2.64, 1/4 1.63 ->
// 1.58, 1/8 1.045 -> 1.03. A/B switch MIINT_T2D_SH (even: kStageRows rows per pass).
#ifndef MIINT_T2D_SH
#define MIINT_T2D_SH 30
#endif
constexpr int kSH = MIINT_T2D_SH;
static_assert(kSH % 2 == 0 && kSH >= 16, "kSH: even, >= the short tile");
// the multi-step row loop's LDS read-ahead (t2d_stream_rows<true>); A/B switch
#ifndef MIINT_T2D_READ_AHEAD
#define MIINT_T2D_READ_AHEAD 1
#endif
// A launch whose row footprint fits half of it stages a kSH / 2-row tile instead: the
// branch-free staging loads every tile row whatever the footprint, so the short footprints of
// the 4-rows-per-wave shapes (multi-GPU row slices) load and write half the rows
// (profiles/r2/table2d_short_tile.jsonl).
constexpr int kSHShort = 16;

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long bits = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(bits), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), lane);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}

// fma(a, s, c) with s in an SGPR pair as one VOP3 v_fma_f64: left to itself hipcc emits
// v_mov_b64 + v_fmac_f64 (c is still live), 3 VALU per sample instead of 2.
__device__ __forceinline__ double fma_sv(double a, double s, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(c));
  return r;
}

// fma(a, b, c) as a 3-operand VOP3 v_fma_f64 with every source a VGPR: left to itself hipcc
// picks the 2-operand v_fmac_f64 (destination tied to c), and a loop-carried result then
// needs a v_mov_b64 from c's register to the value's home; the untied form can be written
// straight there.
__device__ __forceinline__ double fma_vvv(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// One workgroup's share of a row-stream integration, in three parts: its table footprint
// (t2d_footprint), the staging loads of that footprint (t2d_stage_load: SH / kStageRows doubles per
// thread, in registers) and their LDS writes (t2d_stage_store), then the rows
// (t2d_stream_rows). table2d_stream_block runs them in that order for one integration; the
// multi-step kernel issues the NEXT step's staging loads before this step's rows, so their
// latency hides behind the row loop.
struct T2DFoot {
  double sx, sy, cx, cy;
  int c0, r0, r1, tx0, ty0, tx1, ty1;
  int sy0;  // first staged table row: ty0, moved up at the table's bottom edge so that all
            // SH staged rows lie inside it (the tile's row j is table row sy0 + j)
};

__device__ __forceinline__ T2DFoot t2d_footprint(const Table2DParams& p, int rows_per_wave,
                                                 int bx, int by) {
  T2DFoot f;
  f.sx = p.X / p.gx;
  f.sy = p.Y / p.gy;
  f.cx = (p.nx - 1) / p.X;
  f.cy = (p.ny - 1) / p.Y;
  f.c0 = bx * (kWave * kSCols);
  f.r0 = p.row0 + by * (4 * rows_per_wave);
  f.r1 = min(f.r0 + 4 * rows_per_wave, p.row1);
  // table footprint of the workgroup's samples (first / last column and row)
  // (computed on the VALU: readfirstlane moves the uniform results to SGPRs, so the staging
  // addresses below are an SGPR base plus 32-bit lane offsets)
  const int clast = min(f.c0 + kWave * kSCols, p.gx) - 1;
  f.tx0 = __builtin_amdgcn_readfirstlane(
      clampi(static_cast<int>(((f.c0 + 0.5) * f.sx) * f.cx), 0, p.nx - 2));
  f.ty0 = __builtin_amdgcn_readfirstlane(
      clampi(static_cast<int>(((f.r0 + 0.5) * f.sy) * f.cy), 0, p.ny - 2));
  f.tx1 = __builtin_amdgcn_readfirstlane(
      clampi(static_cast<int>(((clast + 0.5) * f.sx) * f.cx), 0, p.nx - 2) + 1);
  f.ty1 = __builtin_amdgcn_readfirstlane(
      clampi(static_cast<int>(((f.r1 - 1 + 0.5) * f.sy) * f.cy), 0, p.ny - 2) + 1);
  f.sy0 = f.ty0;
  return f;
}
template <int SH>
__device__ __forceinline__ void t2d_stage_rows(const Table2DParams& p, T2DFoot& f) {
  f.sy0 = min(f.ty0, p.ny - SH);  // the stream shape needs ny >= SH (table2d_shape)
}

// kSW consecutive lanes per table row, 2 rows per pass; every pass's load in flight before
// the LDS writes. Branch-free, and one lane offset for every pass: SH whole table rows from
// sy0 (inside the table: t2d_stage_rows), a lane right of the footprint loading its last
// column again (same cache line; its LDS slot is never read). Buffer loads: the table's
// resource in SGPRs, the one lane offset in a VGPR and each pass's row offset in an SGPR
// (soffset) — no per-pass address arithmetic on the VALU and no per-pass address VGPRs (a
// global / flat load would take a 64-bit VGPR address per pass: 15 v_lshl_add_u64 and 30
// VGPRs a step).
constexpr int kStageRows = kB / kSW;
// buffer resource word 3 on gfx9 (CDNA): raw (untyped) access, 32-bit data format
constexpr int kBufferRsrcWord3 = 0x00020000;
template <int SH>
__device__ __forceinline__ void t2d_stage_load(const double* table, int nx, int ny,
                                               const T2DFoot& f, double (&v)[SH / kStageRows]) {
  const int w = f.tx1 - f.tx0 + 1;
  const int lx = threadIdx.x % kSW, ly = threadIdx.x / kSW;
  const unsigned off = static_cast<unsigned>(ly * nx + min(lx, w - 1)) * 8u;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(table), static_cast<short>(0), nx * ny * 8, kBufferRsrcWord3);
#pragma unroll
  for (int j = 0; j < SH / kStageRows; ++j) {
    const int soff = ((f.sy0 + kStageRows * j) * nx + f.tx0) * 8;
    v[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, soff, 0));
  }
}

// POISON (validation instantiation, set_lds_poison): tile slots outside the computed
// footprint hold NaN instead of the corner value, so a read outside the footprint shows.
template <int SH, bool POISON>
__device__ __forceinline__ void t2d_stage_store(const T2DFoot& f, const double (&v)[SH / kStageRows],
                                                double* tile) {
  const int lx = threadIdx.x % kSW, ly = threadIdx.x / kSW;
#pragma unroll
  for (int j = 0; j < SH / kStageRows; ++j) tile[(ly + kStageRows * j) * kSW + lx] = v[j];
  if constexpr (POISON) {
    const int w = f.tx1 - f.tx0 + 1;
#pragma unroll
    for (int j = 0; j < SH / kStageRows; ++j) {
      const int row = f.sy0 + ly + kStageRows * j;
      if (!(lx < w && row >= f.ty0 && row <= f.ty1))
        tile[(ly + kStageRows * j) * kSW + lx] = __builtin_nan("");
    }
  }
}

// The rows of the workgroup's block from the staged tile (the barrier before them makes every
// thread's tile writes visible). Returns the block's partial in thread 0.
// READ_AHEAD (the multi-step kernel): the next table row's LDS pair is read one row change
// ahead (below). The single-launch kernels keep the plain read: the read-ahead's 16 extra
// VGPRs would cost them a wave per SIMD (6 -> 5 on the short tile).
template <bool READ_AHEAD = false>
__device__ __forceinline__ double t2d_stream_rows(const Table2DParams& p, int rows_per_wave,
                                                  const T2DFoot& f, const double* tile,
                                                  double* red) {
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int lane = static_cast<int>(threadIdx.x) % kWave;
  // per-lane columns: LDS column and x fraction, computed once
  int col[kSCols];
  double fx[kSCols];
  bool ok[kSCols];
#pragma unroll
  for (int b = 0; b < kSCols; ++b) {
    const int c = f.c0 + lane + kWave * b;
    ok[b] = c < p.gx;
    const double xx = ((min(c, p.gx - 1) + 0.5) * f.sx) * f.cx;
    const int ix = clampi(static_cast<int>(xx), 0, p.nx - 2);
    fx[b] = xx - ix;
    col[b] = ix - f.tx0;
  }
  // this wave's rows; lane k holds row k's table row and fraction
  const int rbase = f.r0 + wave * rows_per_wave;
  const int nrows = max(0, min(rows_per_wave, f.r1 - rbase));
  int iyl;
  double fyl;
  {
    const int r = rbase + min(lane, max(nrows - 1, 0));
    const double yy = ((r + 0.5) * f.sy) * f.cy;
    iyl = clampi(static_cast<int>(yy), 0, p.ny - 2);
    fyl = yy - iyl;
  }
  __syncthreads();
  auto line = [&](int j, int b) {  // table row j interpolated at column b's x
    const double* t = tile + (j - f.sy0) * kSW + col[b];
    // (the untied form only where it removes copies: the single-launch kernels would pay
    // its registers in occupancy)
    if constexpr (READ_AHEAD) return fma_vvv(t[1] - t[0], fx[b], t[0]);
    else return fma(t[1] - t[0], fx[b], t[0]);
  };
  double acc[kSCols], lc[kSCols], ln[kSCols], d[kSCols];
#pragma unroll
  for (int b = 0; b < kSCols; ++b) acc[b] = lc[b] = ln[b] = d[b] = 0.0;
  int cur = -2;
  // The next table row's LDS pair is read one row change ahead: in flight across the rows
  // until the change that needs it, instead of waited for at the change (clamped to the
  // footprint's last row; a read past the rows the wave uses is staged but never used).
  // 4096^2: 5.99 -> 5.86 us per integration, row slices unchanged (profiles/r4/t2d_pf_ab_*).
  double n0[kSCols], n1[kSCols];
  auto fetch = [&](int j) {
#pragma unroll
    for (int b = 0; b < kSCols; ++b) {
      const double* t = tile + (min(j, f.ty1) - f.sy0) * kSW + col[b];
      n0[b] = t[0];
      n1[b] = t[1];
    }
  };
  // Where the table row changes, as two wave-uniform bit masks (one ballot each, once per
  // integration): row k starts a new table row (iy_k != iy_{k-1}; row 0 always), and does so
  // by one (iy_k == iy_{k-1} + 1). The row loop then tests a bit (SALU) instead of reading
  // row k's iy back with a v_readlane every row; iy is read only for the rare jump.
  uint64_t changed, consec;
  {
    const int r = rbase + min(lane, max(nrows - 1, 0));
    const double yyp = ((r - 1 + 0.5) * f.sy) * f.cy;  // row k - 1's, the same arithmetic
    const int iyp = clampi(static_cast<int>(yyp), 0, p.ny - 2);
    changed = __ballot(lane == 0 || iyl != iyp);
    consec = __ballot(lane != 0 && iyl == iyp + 1);
  }
  for (int k = 0; k < nrows; ++k) {
    const double fy = readlane_f64(fyl, k);
    if ((changed >> k) & 1) {  // wave-uniform
      const bool by_one = (consec >> k) & 1;
      const int iy = by_one ? cur + 1 : __builtin_amdgcn_readlane(iyl, k);
      if constexpr (READ_AHEAD) {
        // One path for both kinds of change (one join, so the line values need no phi copies
        // between two predecessors): a jump first sets up what a step by one would hold —
        // ln = line(iy) and the read-ahead at row iy + 1 — and the common update below then
        // forms line(iy + 1) from it exactly as line() does (the same fma).
        if (!by_one) {
#pragma unroll
          for (int b = 0; b < kSCols; ++b) ln[b] = line(iy, b);
          fetch(iy + 1);
        }
#pragma unroll
        for (int b = 0; b < kSCols; ++b) {
          lc[b] = ln[b];
          ln[b] = fma_vvv(n1[b] - n0[b], fx[b], n0[b]);  // line(iy + 1)
          d[b] = ln[b] - lc[b];
        }
        fetch(iy + 2);
      } else if (by_one) {
#pragma unroll
        for (int b = 0; b < kSCols; ++b) {
          lc[b] = ln[b];
          ln[b] = line(iy + 1, b);
          d[b] = ln[b] - lc[b];
        }
      } else {
#pragma unroll
        for (int b = 0; b < kSCols; ++b) {
          lc[b] = line(iy, b);
          ln[b] = line(iy + 1, b);
          d[b] = ln[b] - lc[b];
        }
      }
      cur = iy;
    }
#pragma unroll
    for (int b = 0; b < kSCols; ++b) acc[b] += fma_sv(d[b], fy, lc[b]);
  }
  double a = 0.0;
#pragma unroll
  for (int b = 0; b < kSCols; ++b) a += ok[b] ? acc[b] : 0.0;
  return block_sum<kB>(a, red) * (f.sx * f.sy);
}

// One workgroup's share of a row-stream integration: column block bx, row block by (the
// launch's blockIdx, or the multi-step kernel's). Returns the block's partial in thread 0.
// `between` runs while the staging loads are in flight (the chained close: the loads hold 32
// VGPRs; the kernel is LDS-limited to 4 waves per SIMD, whose 128-VGPR budget the close's 16
// loads in flight fit beside them).
template <int SH, bool POISON, class Between>
__device__ __forceinline__ double table2d_stream_block(const Table2DParams& p, int rows_per_wave,
                                                       int bx, int by, double* tile, double* red,
                                                       Between between) {
  T2DFoot f = t2d_footprint(p, rows_per_wave, bx, by);
  t2d_stage_rows<SH>(p, f);
  double v[SH / kStageRows];
  t2d_stage_load<SH>(p.table, p.nx, p.ny, f, v);
  between();
  t2d_stage_store<SH, POISON>(f, v, tile);
  return t2d_stream_rows(p, rows_per_wave, f, tile, red);
}

template <int MODE, int SH, bool POISON>
__global__ __launch_bounds__(kB) void table2d_stream_kernel(Table2DParams p, int rows_per_wave,
                                                            double* partials, unsigned* ticket,
                                                            double* out, Table2DChain chain) {
  __shared__ double tile[SH * kSW];
  __shared__ double red[kB / kWave];
  __shared__ int is_last;
  const double s = table2d_stream_block<SH, POISON>(
      p, rows_per_wave, blockIdx.x, blockIdx.y, tile, red, [&] {
        if constexpr (MODE == kT2Chained) {
          if (chain.prev && blockIdx.x == 0 && blockIdx.y == 0)
            table2d_close(chain.prev, chain.prev_n, chain.prev_out, red);
        }
      });
  const unsigned bid = blockIdx.y * gridDim.x + blockIdx.x;
  if constexpr (MODE != kT2Fused) {
    if (threadIdx.x == 0) partials[bid] = s;
  } else {
    const unsigned nb = gridDim.x * gridDim.y;
    if (!publish_and_ticket(s, partials, ticket, bid, nb, &is_last)) return;
    const double v = ordered_partials<kB, true>(partials, static_cast<int>(nb));
    rearm_slots<kB>(partials, static_cast<int>(nb));
    const double tot = block_sum<kB>(v, red);
    if (threadIdx.x == 0) out[0] = tot;
    rearm_ticket(ticket, nb);
  }
}

// Multi-step row stream (Table2DConfig::multistep): `steps` complete integrations in one
// launch of resident workgroups (a 1-D grid of the stream shape's gx x gy blocks, block b =
// column block b % gx, row block b / gx: the same linear index as the 2-D launch). Each step
// stages its table footprint again and writes partials[step][b]; multistep_close sums every
// step's partials in index order — bitwise the chained / fused value. One launch ramp and
// tail per replay instead of per integration. The table pointer is laundered through an empty
// asm every step, so no step's loads or arithmetic can be hoisted or shared.
// Step phases (kernels.hpp): the grid is nb x phases workgroups; workgroup g runs block
// g % nb for the steps g / nb, g / nb + phases, ...
// MIINT_T2D_WAVES (A/B): ask the compiler for that many waves per SIMD (register budget)
#ifndef MIINT_T2D_WAVES
#define MIINT_T2D_WAVES 0
#endif
#if MIINT_T2D_WAVES > 0
#define MIINT_T2D_MS_ATTR __attribute__((amdgpu_waves_per_eu(MIINT_T2D_WAVES, 8)))
#else
#define MIINT_T2D_MS_ATTR
#endif
template <int SH>
__global__ __launch_bounds__(kB) MIINT_T2D_MS_ATTR void table2d_multistep_kernel(Table2DParams p, int rows_per_wave,
                                                               int gx, double* partials,
                                                               int steps, unsigned nb) {
  __shared__ double tile[SH * kSW];
  __shared__ double red[kB / kWave];
  const unsigned blk = blockIdx.x % nb;
  const int phases = static_cast<int>(gridDim.x / nb);
  const int first = static_cast<int>(blockIdx.x / nb);
  const int bx = static_cast<int>(blk) % gx, by = static_cast<int>(blk) / gx;
  T2DFoot f = t2d_footprint(p, rows_per_wave, bx, by);
  t2d_stage_rows<SH>(p, f);
  // Each step loads its own footprint from a table pointer laundered per step (no step's
  // loads are shared or hoisted). Short tiles (the multi-GPU row slices): step st's loads are
  // issued during step st - 1, before its rows, so their latency hides behind the row loop
  // (1/8 slice 2.20 -> 2.04 us, profiles/r3/t2d_prefetch_ab.jsonl). The full tile keeps
  // loading at the top of its step: holding its 16 loads across the rows takes 139 VGPRs, 3
  // waves per SIMD, and the 4096^2 grid would no longer be resident.
#ifndef MIINT_T2D_PREFETCH_FULL
#define MIINT_T2D_PREFETCH_FULL 0
#endif
  constexpr bool kPrefetch = SH <= kSHShort || MIINT_T2D_PREFETCH_FULL;
  double v[SH / kStageRows];
  auto load = [&] {
    const double* t = p.table;
    asm volatile("" : "+s"(t));  // a fresh pointer every step (no instructions)
    t2d_stage_load<SH>(t, p.nx, p.ny, f, v);
  };
  if constexpr (kPrefetch) {
    if (first < steps) load();
  }
  for (int st = first; st < steps; st += phases) {
    if constexpr (!kPrefetch) load();
    t2d_stage_store<SH, false>(f, v, tile);
    if constexpr (kPrefetch) {
      if (st + phases < steps) load();
    }
    const double val = t2d_stream_rows<MIINT_T2D_READ_AHEAD != 0>(p, rows_per_wave, f, tile, red);
    if (threadIdx.x == 0) partials[static_cast<size_t>(st) * nb + blk] = val;
    __syncthreads();  // the next step rewrites tile and red
  }
}

__global__ __launch_bounds__(kB) void table2d_multistep_close_kernel(const double* partials,
                                                                     int nb, double* outs) {
  __shared__ double red[kB / kWave];
  table2d_close(partials + static_cast<size_t>(blockIdx.x) * nb, nb, outs + blockIdx.x, red);
}

}  // namespace

// ============================================================================ host side
// One workgroup per CU: the 144 MB re-read (sum + finalize) measured 23.3 us at 256
// workgroups, 23.9 at 512, 25.4 at 1024 = 4 per CU, the earlier default
// (profiles/r2/sum_array_grid.jsonl).
int default_reduce_grid(int num_cus) { return num_cus; }

void launch_sum_array(const double* x, uint64_t n, double scale, double* partials, int grid,
                      double* out, hipStream_t stream) {
  MIINT_CHECK(n >= 1 && grid >= 1, "empty sum");
  MIINT_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0, "sum_array needs 16-B alignment");
  sum_array_kernel<<<grid, kB, 0, stream>>>(x, n, partials);
  MIINT_HIP(hipGetLastError());
  launch_finalize(partials, grid, scale, out, stream);
}

void set_lds_poison_table(bool on) {
  const int v = on ? 1 : 0;
  MIINT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_lds_poison), &v, sizeof(v)));
  g_table2d_poison.store(on);
}

void set_lds_poison(bool on) {
  set_lds_poison_table(on);
  set_lds_poison_trainscan(on);
}

void launch_interp_fill(const double* table, int table_n, double dt, uint64_t i0, uint64_t n,
                        double* y, hipStream_t stream) {
  MIINT_CHECK(table_n >= 2 && table_n <= kMaxTable, "table size must be in [2, 2048]");
  MIINT_CHECK((reinterpret_cast<uintptr_t>(y) & 15) == 0, "interp_fill needs 16-B alignment");
  MIINT_CHECK(n >= 1, "empty fill");
  MIINT_CHECK(dt > 0.0 && std::isfinite(dt), "interp_fill needs a finite dt > 0");
  // 2048 workgroups = 8 waves on each of the 256 CUs' 4 SIMDs; chunks a multiple of 256
  // vectors so every pass but a chunk's last stores whole 4 KB lines
  const uint64_t nv = n / 2;
  const uint64_t per = (nv + kFillBlocks - 1) / kFillBlocks;
  const uint64_t chunk = std::max<uint64_t>(kB, (per + kB - 1) / kB * kB);
  const int grid = static_cast<int>(std::max<uint64_t>(1, (nv + chunk - 1) / chunk));
  interp_fill_kernel<<<grid, kB, 0, stream>>>(table, table_n, dt, i0, n, chunk, y);
  MIINT_HIP(hipGetLastError());
}

void launch_outer_product(const double* v, int n, double* table, hipStream_t stream) {
  MIINT_CHECK(n >= 1 && n <= 65535, "outer product size");
  outer_product_kernel<<<dim3((n + kB - 1) / kB, n), kB, 0, stream>>>(v, n, table);
  MIINT_HIP(hipGetLastError());
}

// Launch shape. Row stream when a workgroup's footprint (256 columns x 4 R rows) fits the
// kSW x kSH LDS tile, with R (rows per wave) the largest of 32, 16, 8, 4 that fits and
// still gives at least 512 workgroups (else the smallest that fits). Measured on 4096^2 and
// 8192^2 fields and their 1/2, 1/4, 1/8 row slices: more rows per lane beat more
// workgroups down to ~512 of them (profiles/r1/table2d_stream_rows.jsonl). Otherwise the
// tile kernel, 128-sample tiles unless that leaves fewer than 4 per CU (1024).
namespace {
struct Table2DShape {
  bool stream;
  bool short_tile;    // stream: the footprint fits kSHShort rows
  int rows_per_wave;  // stream
  int tile;           // tile kernel: 128 or 64
  dim3 grid;
};

Table2DShape table2d_shape(const Table2DParams& p) {
  const double step_x = (p.X / p.gx) * ((p.nx - 1) / p.X);  // cells per sample
  const double step_y = (p.Y / p.gy) * ((p.ny - 1) / p.Y);
  const int rows = p.row1 - p.row0;
  const int gxs = (p.gx + kWave * kSCols - 1) / (kWave * kSCols);
  Table2DShape sh{};
  // table cells n samples touch: their first and last cells floor(a), floor(a + (n-1) step)
  // are at most floor((n-1) step) + 1 apart, + 1 for the last one's +1 neighbour (the
  // 1e-9 guards a product that lands a rounding below an integer)
  auto span = [](int n, double step) { return std::floor((n - 1) * step + 1e-9) + 3.0; };
  // (a staged tile is SH whole table rows: the table needs at least that many)
  if (span(kWave * kSCols, step_x) <= kSW && p.ny >= kSHShort) {
    for (int r : {32, 16, 8, 4}) {
      if (span(4 * r, step_y) > (p.ny >= kSH ? kSH : kSHShort)) continue;
      const long nwg = static_cast<long>(gxs) * ((rows + 4 * r - 1) / (4 * r));
      sh.stream = true;
      sh.rows_per_wave = r;
      sh.short_tile = span(4 * r, step_y) <= kSHShort;
      sh.grid = dim3(gxs, (rows + 4 * r - 1) / (4 * r));
      if (nwg >= (p.min_wg > 0 ? p.min_wg : 512)) break;
    }
    if (sh.stream) return sh;
  }
  const long t128 = static_cast<long>((p.gx + 127) / 128) * ((rows + 127) / 128);
  sh.tile = t128 >= 1024 ? 128 : 64;
  sh.grid = dim3((p.gx + sh.tile - 1) / sh.tile, (rows + sh.tile - 1) / sh.tile);
  return sh;
}
}  // namespace

int table2d_grid(const Table2DParams& p) {
  const Table2DShape sh = table2d_shape(p);
  return static_cast<int>(sh.grid.x * sh.grid.y);
}

Table2DShapeInfo table2d_shape_info(const Table2DParams& p) {
  const Table2DShape sh = table2d_shape(p);
  return {sh.stream, sh.stream ? sh.rows_per_wave : 0,
          sh.stream ? (sh.short_tile ? kSHShort : kSH) : 0, sh.stream ? kSW : 0,
          static_cast<int>(sh.grid.x), static_cast<int>(sh.grid.y), sh.stream ? 0 : sh.tile};
}

const char* table2d_path(const Table2DParams& p) {
  const Table2DShape sh = table2d_shape(p);
  return sh.stream ? "stream" : "tile";
}

static void check_table2d(const Table2DParams& p) {
  MIINT_CHECK(p.nx >= 2 && p.ny >= 2 && p.gx >= 1 && p.gy >= 1, "table2d dims");
  // the row stream's buffer loads address the table with 32-bit byte offsets
  MIINT_CHECK(static_cast<long long>(p.nx) * p.ny * 8 < (1LL << 31), "table2d: table over 2 GB");
  MIINT_CHECK(p.row0 >= 0 && p.row1 <= p.gy && p.row0 < p.row1, "table2d row range");
}

template <int MODE>
static void launch_table2d(const Table2DParams& p, double* partials, unsigned* ticket,
                           double* out, Table2DChain chain, hipStream_t stream) {
  check_table2d(p);
  const Table2DShape sh = table2d_shape(p);
  const bool poison = g_table2d_poison.load(std::memory_order_relaxed);
  if (sh.stream && sh.short_tile && poison)
    table2d_stream_kernel<MODE, kSHShort, true><<<sh.grid, kB, 0, stream>>>(
        p, sh.rows_per_wave, partials, ticket, out, chain);
  else if (sh.stream && sh.short_tile)
    table2d_stream_kernel<MODE, kSHShort, false><<<sh.grid, kB, 0, stream>>>(
        p, sh.rows_per_wave, partials, ticket, out, chain);
  else if (sh.stream && poison)
    table2d_stream_kernel<MODE, kSH, true><<<sh.grid, kB, 0, stream>>>(
        p, sh.rows_per_wave, partials, ticket, out, chain);
  else if (sh.stream)
    table2d_stream_kernel<MODE, kSH, false><<<sh.grid, kB, 0, stream>>>(
        p, sh.rows_per_wave, partials, ticket, out, chain);
  else if (sh.tile == 128)
    table2d_kernel<128, MODE><<<sh.grid, kB, 0, stream>>>(p, partials, ticket, out, chain);
  else
    table2d_kernel<64, MODE><<<sh.grid, kB, 0, stream>>>(p, partials, ticket, out, chain);
  MIINT_HIP(hipGetLastError());
}

void launch_table2d_partials(const Table2DParams& p, double* partials, hipStream_t stream) {
  launch_table2d<kT2Partials>(p, partials, nullptr, nullptr, {nullptr, 0, nullptr}, stream);
}

void launch_table2d_fused(const Table2DParams& p, double* partials, unsigned* ticket,
                          double* out, hipStream_t stream) {
  launch_table2d<kT2Fused>(p, partials, ticket, out, {nullptr, 0, nullptr}, stream);
}

void launch_table2d_chained(const Table2DParams& p, double* partials, const double* prev,
                            double* prev_out, hipStream_t stream) {
  MIINT_CHECK(prev == nullptr || prev_out != nullptr, "chained table2d: prev without prev_out");
  MIINT_CHECK(prev == nullptr || prev != partials, "chained table2d: prev aliases partials");
  const int nb = table2d_grid(p);
  launch_table2d<kT2Chained>(p, partials, nullptr, nullptr, {prev, nb, prev_out}, stream);
}

namespace {
template <int SH>
int t2d_ms_per_cu() {
  int n = 0;
  MIINT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &n, reinterpret_cast<const void*>(&table2d_multistep_kernel<SH>), kB, 0));
  return n;
}
}  // namespace

int table2d_multistep_resident(const Table2DParams& p) {
  check_table2d(p);
  const Table2DShape sh = table2d_shape(p);
  if (!sh.stream) return 0;
  return sh.short_tile ? t2d_ms_per_cu<kSHShort>() : t2d_ms_per_cu<kSH>();
}

bool table2d_multistep_ok(const Table2DParams& p, int num_cus) {
  return table2d_multistep_phases(p, num_cus, 1) >= 1;
}

// Step phases for a launch of `steps`: 0 if the shape is not the row stream; else `want` (an
// explicit request) or, for want = 0, kT2AutoPhases — both capped by steps (and an explicit
// one by kT2MaxPhases). Residency is not required: the kernel's workgroups never wait on each
// other, and past it the multi-step replay still beats chained launches
// (profiles/r4/t2d_ms_any_ab.jsonl: 6144^2 10.5 -> 9.15 us, 8192^2 13.3 -> 12.2 us, where
// not one phase is resident).
int table2d_multistep_phases(const Table2DParams& p, int num_cus, int steps, int want) {
  check_table2d(p);
  (void)num_cus;
  if (!table2d_shape(p).stream) return 0;
  // Past residency the later phases' workgroups start as earlier ones finish (each runs
  // steps / phases steps): more phases won or tied everywhere measured, up to 16
  // (profiles/r4/t2d_phases_explicit.jsonl, t2d_variant_ab.jsonl, t2d_shape_sweep.jsonl, us
  // per integration; 4096^2: 5.87 / 5.56 / 5.39 / 5.36 at 1-4 phases on 32-row tiles, 5.13 /
  // 5.07 at 8 / 16 on 30-row tiles; the 1/8 slice 1.92 / 1.48 / 1.49 / 1.45, then 1.01 / 0.97)
  // Auto also doubles the phases (up to kT2MaxPhases) while a replay would run fewer than
  // kT2AutoWorkgroups workgroups: the 1/8 slice's 128 blocks at 1024 integrations per replay,
  // 0.61 -> 0.58 us at 32 phases; the whole field (1024 blocks) ran slower at 32 (4.14-4.30 ->
  // 4.31-4.49 us; profiles/r5/t2d/n_t2d_steps.jsonl).
  int phases = kT2AutoPhases;
  if (want > 0) {
    phases = std::min(want, kT2MaxPhases);
  } else {
    const long nb = static_cast<long>(table2d_grid(p));
    while (phases < kT2MaxPhases && nb * phases < kT2AutoWorkgroups) phases *= 2;
  }
  return std::min(phases, std::max(1, steps));
}

void launch_table2d_multistep(const Table2DParams& p, double* partials, int steps, double* outs,
                              hipStream_t stream, int phases) {
  check_table2d(p);
  MIINT_CHECK(steps >= 1 && steps <= 1024, "table2d multi-step: 1..1024 steps");
  MIINT_CHECK(phases >= 1 && phases <= kT2MaxPhases, "table2d multi-step: 1..kT2MaxPhases step phases");
  const Table2DShape sh = table2d_shape(p);
  MIINT_CHECK(sh.stream, "table2d multi-step runs the row-stream shape only");
  const int nb = static_cast<int>(sh.grid.x * sh.grid.y);
  const int gx = static_cast<int>(sh.grid.x);
  const unsigned grid = static_cast<unsigned>(nb) * static_cast<unsigned>(phases);
  if (sh.short_tile)
    table2d_multistep_kernel<kSHShort><<<grid, kB, 0, stream>>>(p, sh.rows_per_wave, gx, partials,
                                                               steps, static_cast<unsigned>(nb));
  else
    table2d_multistep_kernel<kSH><<<grid, kB, 0, stream>>>(p, sh.rows_per_wave, gx, partials,
                                                          steps, static_cast<unsigned>(nb));
  MIINT_HIP(hipGetLastError());
  table2d_multistep_close_kernel<<<steps, kB, 0, stream>>>(partials, nb, outs);
  MIINT_HIP(hipGetLastError());
}

void launch_table2d_finalize(const double* partials, int n, double* out, hipStream_t stream) {
  MIINT_CHECK(n >= 1, "table2d finalize: no partials");
  table2d_finalize_kernel<<<1, kB, 0, stream>>>(partials, n, out);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
