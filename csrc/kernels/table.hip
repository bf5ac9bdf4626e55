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

#include "miint/common.hpp"
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
// Workgroup = 16x16 threads = one 64x64 tile of sample points (4x4 per thread).
constexpr int kTile = 64;
constexpr int kLdsDim = 48;  // table footprint per tile in LDS: up to 48x48 doubles = 18 KB

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <bool USE_LDS>
__global__ __launch_bounds__(kB) void table2d_kernel(Table2DParams p, double* partials) {
  __shared__ double tile[kLdsDim * (kLdsDim + 1)];
  __shared__ double red[kB / kWave];
  const double sx = p.X / p.gx, sy = p.Y / p.gy;          // sample spacing
  const double cx = (p.nx - 1) / p.X, cy = (p.ny - 1) / p.Y;  // table cells per unit
  const int c0 = blockIdx.x * kTile;
  const int r0 = p.row0 + blockIdx.y * kTile;
  // Table footprint of this tile: cells touched by its first and last sample.
  const int tx0 = clampi(static_cast<int>(((c0 + 0.5) * sx) * cx), 0, p.nx - 2);
  const int ty0 = clampi(static_cast<int>(((r0 + 0.5) * sy) * cy), 0, p.ny - 2);
  if constexpr (USE_LDS) {
    const int tx1 = clampi(static_cast<int>(((c0 + kTile - 0.5) * sx) * cx), 0, p.nx - 2) + 1;
    const int ty1 = clampi(static_cast<int>(((r0 + kTile - 0.5) * sy) * cy), 0, p.ny - 2) + 1;
    const int w = tx1 - tx0 + 1, hgt = ty1 - ty0 + 1;
    for (int k = threadIdx.x; k < w * hgt; k += kB) {
      const int rr = k / w, cc = k - rr * w;
      tile[rr * (kLdsDim + 1) + cc] = p.table[static_cast<size_t>(ty0 + rr) * p.nx + tx0 + cc];
    }
    __syncthreads();
  }
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int r = r0 + ty + 16 * a;
    if (r >= p.row1) break;
    const double yy = ((r + 0.5) * sy) * cy;
    const int iy = clampi(static_cast<int>(yy), 0, p.ny - 2);
    const double fy = yy - iy;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = c0 + tx + 16 * b;
      if (c >= p.gx) break;
      const double xx = ((c + 0.5) * sx) * cx;
      const int ix = clampi(static_cast<int>(xx), 0, p.nx - 2);
      const double fx = xx - ix;
      double v00, v01, v10, v11;
      if constexpr (USE_LDS) {
        const double* t = tile + (iy - ty0) * (kLdsDim + 1) + (ix - tx0);
        v00 = t[0]; v01 = t[1]; v10 = t[kLdsDim + 1]; v11 = t[kLdsDim + 2];
      } else {
        const double* t = p.table + static_cast<size_t>(iy) * p.nx + ix;
        v00 = t[0]; v01 = t[1]; v10 = t[p.nx]; v11 = t[p.nx + 1];
      }
      const double top = fma(v01 - v00, fx, v00);
      const double bot = fma(v11 - v10, fx, v10);
      acc += fma(bot - top, fy, top);
    }
  }
  const double s = block_sum<kB>(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = s * (sx * sy);
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

static bool table2d_fits_lds(const Table2DParams& p) {
  // cells spanned by kTile samples (+2 for partial cells at both ends)
  const double cells_x = kTile * (p.X / p.gx) * ((p.nx - 1) / p.X) + 2.0;
  const double cells_y = kTile * (p.Y / p.gy) * ((p.ny - 1) / p.Y) + 2.0;
  return cells_x + 1.0 <= kLdsDim && cells_y + 1.0 <= kLdsDim;
}

int table2d_grid(const Table2DParams& p) {
  const int gxb = (p.gx + kTile - 1) / kTile;
  const int gyb = (p.row1 - p.row0 + kTile - 1) / kTile;
  return gxb * gyb;
}

void launch_table2d_partials(const Table2DParams& p, double* partials, hipStream_t stream) {
  MIINT_CHECK(p.nx >= 2 && p.ny >= 2 && p.gx >= 1 && p.gy >= 1, "table2d dims");
  MIINT_CHECK(p.row0 >= 0 && p.row1 <= p.gy && p.row0 < p.row1, "table2d row range");
  const dim3 grid((p.gx + kTile - 1) / kTile, (p.row1 - p.row0 + kTile - 1) / kTile);
  if (table2d_fits_lds(p)) table2d_kernel<true><<<grid, kB, 0, stream>>>(p, partials);
  else table2d_kernel<false><<<grid, kB, 0, stream>>>(p, partials);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
