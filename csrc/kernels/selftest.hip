// Self-test kernels exposing the wave/block primitives of wave_reduce.hpp on raw arrays,
// so tests can check the DPP reductions and scans against a plain fp64/fp32 reference
// (including partial waves and 1..16-wave workgroups, SURVEY §7.4 "reduction tests").
#include <hip/hip_runtime.h>

#include "miint/common.hpp"
#include "miint/selftest.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {
namespace {

// Per-wave sum and inclusive scan of `in` (n elements, zero-padded to whole waves).
template <typename T>
__global__ __launch_bounds__(256) void wave_ops_kernel(const T* in, uint64_t n, T* wave_sums,
                                                       T* scan) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  const T v = i < n ? in[i] : T(0);
  const T s = wave_sum(v);
  const T c = wave_inclusive_scan(v);
  if (i < n) scan[i] = c;
  if ((threadIdx.x & 63) == 0 && i < n) wave_sums[i / 64] = s;
}

// Block sum / block scan with a compile-time block size.
template <int BLOCK, typename T>
__global__ __launch_bounds__(BLOCK) void block_ops_kernel(const T* in, uint64_t n, T* block_sums,
                                                          T* scan) {
  __shared__ T red[BLOCK / kWave];
  __shared__ T red2[BLOCK / kWave];
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * BLOCK + threadIdx.x;
  const T v = i < n ? in[i] : T(0);
  const T s = block_sum<BLOCK>(v, red);
  T total;
  const T c = block_inclusive_scan<BLOCK>(v, red2, &total);
  if (i < n) scan[i] = c;
  if (threadIdx.x == 0) block_sums[blockIdx.x] = s;
}

template <typename T>
void wave_ops_t(const T* in, uint64_t n, T* sums, T* scan, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>((n + 255) / 256);
  wave_ops_kernel<T><<<grid, 256, 0, s>>>(in, n, sums, scan);
}

template <typename T>
void block_ops_t(const T* in, uint64_t n, int block, T* sums, T* scan, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>((n + block - 1) / block);
  switch (block) {
#define MIINT_BLK(Bk) case Bk: block_ops_kernel<Bk, T><<<grid, Bk, 0, s>>>(in, n, sums, scan); break;
    MIINT_BLK(64) MIINT_BLK(128) MIINT_BLK(192) MIINT_BLK(256) MIINT_BLK(512) MIINT_BLK(1024)
#undef MIINT_BLK
    default: fail("block must be one of 64,128,192,256,512,1024", __FILE__, __LINE__);
  }
}

}  // namespace

void selftest_wave_ops(const void* in, uint64_t n, bool f32, void* sums, void* scan,
                       hipStream_t s) {
  MIINT_CHECK(n >= 1, "empty input");
  if (f32) wave_ops_t(static_cast<const float*>(in), n, static_cast<float*>(sums),
                      static_cast<float*>(scan), s);
  else wave_ops_t(static_cast<const double*>(in), n, static_cast<double*>(sums),
                  static_cast<double*>(scan), s);
  MIINT_HIP(hipGetLastError());
}

void selftest_block_ops(const void* in, uint64_t n, int block, bool f32, void* sums, void* scan,
                        hipStream_t s) {
  MIINT_CHECK(n >= 1, "empty input");
  if (f32) block_ops_t(static_cast<const float*>(in), n, block, static_cast<float*>(sums),
                       static_cast<float*>(scan), s);
  else block_ops_t(static_cast<const double*>(in), n, block, static_cast<double*>(sums),
                   static_cast<double*>(scan), s);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
