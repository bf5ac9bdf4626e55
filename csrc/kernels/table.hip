// Table kernels for gfx950: HBM-bound array sum, interpolated-profile fill, and the 2-D
// bilinear field integral.
//
// Reference counterparts:
//   cuda_test pass 1  cintegrate.cu:88-92  d_InterpProfile[i] = faccel(i*dt) — 3 global
//                     loads/sample, per-thread contiguous chunks (uncoalesced stores)
//   cuda_test pass 2  cintegrate.cu:94-96  serial re-read of the 144 MB array per thread
//   4main fill        4main.c:82-86        same fill on the host
// Here: table staged once per workgroup in LDS, 16-byte stores/loads per lane
// (global_store_dwordx4 / global_load_dwordx4), grid-stride over 64-bit indices.
// The 2-D config (BASELINE.json #5) has no reference counterpart: it integrates a
// ny x nx fp64 field with bilinear interpolation, each workgroup staging the table
// footprint of its 64x64 sample tile in LDS (2-D LDS tiling).
#include <hip/hip_runtime.h>

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

__device__ __forceinline__ double interp_lds(const double* tab, int nseg, double t) {
  int i = static_cast<int>(t);
  i = i < 0 ? 0 : (i >= nseg ? nseg - 1 : i);
  const double v0 = tab[i];
  return fma(tab[i + 1] - v0, t - static_cast<double>(i), v0);
}

__global__ __launch_bounds__(kB) void interp_fill_kernel(const double* __restrict__ table,
                                                         int table_n, double dt, uint64_t i0,
                                                         uint64_t n, double* __restrict__ y) {
  __shared__ double tab[kMaxTable];
  for (int k = threadIdx.x; k < table_n; k += kB) tab[k] = table[k];
  __syncthreads();
  const int nseg = table_n - 1;
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * kB;
  const uint64_t nv = n / 2;
  f64x2* yv = reinterpret_cast<f64x2*>(y);
  // y may be at an odd element offset inside a larger buffer only if the caller passes
  // an aligned pointer; the launcher checks 16-B alignment.
  for (uint64_t v = static_cast<uint64_t>(blockIdx.x) * kB + threadIdx.x; v < nv; v += lanes) {
    const uint64_t i = i0 + 2 * v;
    f64x2 o;
    o.x = interp_lds(tab, nseg, dt * static_cast<double>(i));
    o.y = interp_lds(tab, nseg, dt * static_cast<double>(i + 1));
    yv[v] = o;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
    y[n - 1] = interp_lds(tab, nseg, dt * static_cast<double>(i0 + n - 1));
}

// ---------------------------------------------------------------------------- outer product
__global__ __launch_bounds__(kB) void outer_product_kernel(const double* __restrict__ v, int n,
                                                           double* __restrict__ t) {
  const int j = blockIdx.x * kB + threadIdx.x;
  const int i = blockIdx.y;
  if (j < n) t[static_cast<size_t>(i) * n + j] = v[i] * v[j];
}

// ---------------------------------------------------------------------------- table2d
// Workgroup = 16 x 16 threads = one TILE x TILE tile of sample points: TILE = 128 (8 x 8 per
// thread) when the grid gives every CU at least 4 such tiles, else TILE = 64 (4 x 4 per
// thread): an 8-GPU row slice of 4096^2 is 128 tiles of 128 for 256 CUs.
// Table footprint per tile in LDS: up to 64 x 64 doubles for 128-sample tiles (33 KB: 4
// workgroups per CU, so a 4096^2 grid is one resident wave), 32 x 32 for 64-sample tiles
// (8.4 KB: the LDS no longer caps residency).
template <int kTile>
constexpr int lds_dim() { return kTile == 128 ? 64 : 32; }

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Per thread: 8 x 8 samples (columns c0 + tx + 16 b, rows r0 + ty + 16 a). The column
// terms (LDS column, fraction) and row terms (LDS row offset, fraction) are computed once
// per thread — 16 index computations instead of 64 (the first form spent 41 VALU per sample,
// SQ_INSTS_VALU 1.07e7 for 16.8e6 samples) — leaving per sample one integer add, two
// ds_read2_b64 and the bilinear blend. FUSED: the last workgroup reduces all partials
// (handoff.hpp) and writes out[0]; otherwise one partial per workgroup for a finalize.
template <int kTile, bool USE_LDS, bool FUSED>
__global__ __launch_bounds__(kB) void table2d_kernel(Table2DParams p, double* partials,
                                                     unsigned* ticket, double* out) {
  constexpr int kPer = kTile / 16;
  constexpr int kLdsDim = lds_dim<kTile>();
  __shared__ double tile[kLdsDim * (kLdsDim + 1)];
  __shared__ double red[kB / kWave];
  __shared__ int is_last;
  const double sx = p.X / p.gx, sy = p.Y / p.gy;          // sample spacing
  const double cx = (p.nx - 1) / p.X, cy = (p.ny - 1) / p.Y;  // table cells per unit
  const int c0 = blockIdx.x * kTile;
  const int r0 = p.row0 + blockIdx.y * kTile;
  // Table footprint of this tile: cells touched by its first and last sample.
  const int tx0 = clampi(static_cast<int>(((c0 + 0.5) * sx) * cx), 0, p.nx - 2);
  const int ty0 = clampi(static_cast<int>(((r0 + 0.5) * sy) * cy), 0, p.ny - 2);
  if constexpr (USE_LDS) {
    // kLdsDim consecutive lanes per table row (coalesced), kRowsPer rows per pass: all
    // passes' loads in flight before the LDS writes (a k / w loop issued them one latency at
    // a time).
    constexpr int kRowsPer = kB / kLdsDim, kPasses = kLdsDim / kRowsPer;
    const int tx1 = clampi(static_cast<int>(((c0 + kTile - 0.5) * sx) * cx), 0, p.nx - 2) + 1;
    const int ty1 = clampi(static_cast<int>(((r0 + kTile - 0.5) * sy) * cy), 0, p.ny - 2) + 1;
    const int w = tx1 - tx0 + 1, hgt = ty1 - ty0 + 1;
    const int lx = threadIdx.x % kLdsDim, ly = threadIdx.x / kLdsDim;
    double v[kPasses];
#pragma unroll
    for (int j = 0; j < kPasses; ++j) {
      const int rr = ly + kRowsPer * j;
      v[j] = (lx < w && rr < hgt) ? p.table[static_cast<size_t>(ty0 + rr) * p.nx + tx0 + lx]
                                  : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kPasses; ++j) tile[(ly + kRowsPer * j) * (kLdsDim + 1) + lx] = v[j];
    __syncthreads();
  }
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  constexpr int kRow = kLdsDim + 1;
  using Off = typename std::conditional<USE_LDS, int, size_t>::type;  // 32-bit LDS offsets
  Off col[kPer], row[kPer];
  double fx[kPer], fy[kPer];
#pragma unroll
  for (int b = 0; b < kPer; ++b) {
    const int c = c0 + tx + 16 * b;
    const double xx = ((c + 0.5) * sx) * cx;
    const int ix = clampi(static_cast<int>(xx), 0, p.nx - 2);
    fx[b] = xx - ix;
    col[b] = USE_LDS ? ix - tx0 : ix;
  }
#pragma unroll
  for (int a = 0; a < kPer; ++a) {
    const int r = r0 + ty + 16 * a;
    const double yy = ((r + 0.5) * sy) * cy;
    const int iy = clampi(static_cast<int>(yy), 0, p.ny - 2);
    fy[a] = yy - iy;
    row[a] = USE_LDS ? static_cast<Off>((iy - ty0) * kRow) : static_cast<Off>(iy) * p.nx;
  }
  const double* base = USE_LDS ? tile : p.table;
  const Off stride = USE_LDS ? static_cast<Off>(kRow) : static_cast<Off>(p.nx);
  auto sample = [&](int a, int b) {
    const double* t = base + (row[a] + col[b]);
    const double v00 = t[0], v01 = t[1], v10 = t[stride], v11 = t[stride + 1];
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
  if constexpr (!FUSED) {
    if (threadIdx.x == 0) partials[bid] = s;
  } else {
    const unsigned nb = gridDim.x * gridDim.y;
    if (!publish_and_ticket(s, partials, ticket, bid, nb, &is_last)) return;
    const double tot = block_sum<kB>(ordered_partials<kB, true>(partials, static_cast<int>(nb)), red);
    if (threadIdx.x == 0) out[0] = tot;
    rearm_ticket(ticket, nb);
  }
}

}  // namespace

// ============================================================================ host side
int default_reduce_grid(int num_cus) { return num_cus * 4; }

void launch_sum_array(const double* x, uint64_t n, double scale, double* partials, int grid,
                      double* out, hipStream_t stream) {
  MIINT_CHECK(n >= 1 && grid >= 1, "empty sum");
  MIINT_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0, "sum_array needs 16-B alignment");
  sum_array_kernel<<<grid, kB, 0, stream>>>(x, n, partials);
  MIINT_HIP(hipGetLastError());
  launch_finalize(partials, grid, scale, out, stream);
}

void launch_interp_fill(const double* table, int table_n, double dt, uint64_t i0, uint64_t n,
                        double* y, hipStream_t stream) {
  MIINT_CHECK(table_n >= 2 && table_n <= kMaxTable, "table size must be in [2, 2048]");
  MIINT_CHECK((reinterpret_cast<uintptr_t>(y) & 15) == 0, "interp_fill needs 16-B alignment");
  MIINT_CHECK(n >= 1, "empty fill");
  const uint64_t nv = (n + 1) / 2;
  const int grid = static_cast<int>(std::min<uint64_t>((nv + kB - 1) / kB, 8192));
  interp_fill_kernel<<<grid, kB, 0, stream>>>(table, table_n, dt, i0, n, y);
  MIINT_HIP(hipGetLastError());
}

void launch_outer_product(const double* v, int n, double* table, hipStream_t stream) {
  MIINT_CHECK(n >= 1 && n <= 65535, "outer product size");
  outer_product_kernel<<<dim3((n + kB - 1) / kB, n), kB, 0, stream>>>(v, n, table);
  MIINT_HIP(hipGetLastError());
}

// Tile edge for this launch: 128 unless that leaves fewer than 4 tiles per CU (1024).
static int table2d_tile(const Table2DParams& p) {
  const long t128 = static_cast<long>((p.gx + 127) / 128) * ((p.row1 - p.row0 + 127) / 128);
  return t128 >= 1024 ? 128 : 64;
}

static bool table2d_fits_lds(const Table2DParams& p, int tile) {
  // cells spanned by `tile` samples (+2 for partial cells at both ends)
  const double cells_x = tile * (p.X / p.gx) * ((p.nx - 1) / p.X) + 2.0;
  const double cells_y = tile * (p.Y / p.gy) * ((p.ny - 1) / p.Y) + 2.0;
  const int dim = tile == 128 ? lds_dim<128>() : lds_dim<64>();
  return cells_x + 1.0 <= dim && cells_y + 1.0 <= dim;
}

int table2d_grid(const Table2DParams& p) {
  const int t = table2d_tile(p);
  const int gxb = (p.gx + t - 1) / t;
  const int gyb = (p.row1 - p.row0 + t - 1) / t;
  return gxb * gyb;
}

static void check_table2d(const Table2DParams& p) {
  MIINT_CHECK(p.nx >= 2 && p.ny >= 2 && p.gx >= 1 && p.gy >= 1, "table2d dims");
  MIINT_CHECK(p.row0 >= 0 && p.row1 <= p.gy && p.row0 < p.row1, "table2d row range");
}

static dim3 table2d_dims(const Table2DParams& p, int t) {
  return dim3((p.gx + t - 1) / t, (p.row1 - p.row0 + t - 1) / t);
}

template <bool FUSED>
static void launch_table2d(const Table2DParams& p, double* partials, unsigned* ticket,
                           double* out, hipStream_t stream) {
  check_table2d(p);
  const int t = table2d_tile(p);
  const dim3 grid = table2d_dims(p, t);
  const bool lds = table2d_fits_lds(p, t);
  if (t == 128) {
    if (lds) table2d_kernel<128, true, FUSED><<<grid, kB, 0, stream>>>(p, partials, ticket, out);
    else table2d_kernel<128, false, FUSED><<<grid, kB, 0, stream>>>(p, partials, ticket, out);
  } else {
    if (lds) table2d_kernel<64, true, FUSED><<<grid, kB, 0, stream>>>(p, partials, ticket, out);
    else table2d_kernel<64, false, FUSED><<<grid, kB, 0, stream>>>(p, partials, ticket, out);
  }
  MIINT_HIP(hipGetLastError());
}

void launch_table2d_partials(const Table2DParams& p, double* partials, hipStream_t stream) {
  launch_table2d<false>(p, partials, nullptr, nullptr, stream);
}

void launch_table2d_fused(const Table2DParams& p, double* partials, unsigned* ticket,
                          double* out, hipStream_t stream) {
  launch_table2d<true>(p, partials, ticket, out, stream);
}

}  // namespace miint
