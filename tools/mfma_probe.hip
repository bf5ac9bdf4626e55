// Microbenchmark: fp64 MFMA throughput on gfx950 and its co-execution with fp64 VALU.
//
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o build/bin/mfma_probe
//   build/bin/mfma_probe
//
// Kernels (one workgroup of 4 waves per CU slot, grid = 256 CUs x 8 workgroups):
//   mfma   : each wave issues ITER v_mfma_f64_16x16x4_f64 on 4 independent accumulators
//   valu   : each wave issues ITER x 16 independent v_fma_f64 (4 chains)
//   mixed  : waves 0,1 of each workgroup run the mfma loop, waves 2,3 the valu loop
// Reports cycles per instruction per SIMD (at the measured clock) to decide whether the
// Pi4 hot loop can move part of its per-sample arithmetic onto the matrix cores.
//
// Result (MI355X, profiles/r1/mfma_probe.json): 58.5 cycles per f64 16x16x4 MFMA per SIMD
// (2048 flops -> the same arithmetic rate as the vector unit), 3.97 per v_fma_f64, and the
// mixed kernel takes 2.92 ms vs 1.83 ms if MFMA and VALU waves overlapped perfectly — they
// nearly serialise. So the fp64 hot loops stay on the VALU.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                         \
  do {                                                                                    \
    hipError_t e = (x);                                                                   \
    if (e != hipSuccess) {                                                                \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));               \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kIter = 4096;

__device__ __forceinline__ void mfma_loop(double a, double b, double* out) {
  f64x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < kIter; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[0] = c0.x + c1.y + c2.z + c3.w;
}

__device__ __forceinline__ void valu_loop(double a, double b, double* out) {
  double x0 = a, x1 = b, x2 = a + 1, x3 = b + 1;
  for (int i = 0; i < kIter; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x0 = fma(x0, a, b);
      x1 = fma(x1, a, b);
      x2 = fma(x2, a, b);
      x3 = fma(x3, a, b);
    }
  }
  out[0] = x0 + x1 + x2 + x3;
}

__global__ __launch_bounds__(256) void k_mfma(double a, double b, double* out) {
  mfma_loop(a, b, out + blockIdx.x * 256 + threadIdx.x);
}
__global__ __launch_bounds__(256) void k_valu(double a, double b, double* out) {
  valu_loop(a, b, out + blockIdx.x * 256 + threadIdx.x);
}
__global__ __launch_bounds__(256) void k_mixed(double a, double b, double* out) {
  if ((threadIdx.x >> 6) < 2) mfma_loop(a, b, out + blockIdx.x * 256 + threadIdx.x);
  else valu_loop(a, b, out + blockIdx.x * 256 + threadIdx.x);
}

template <class K>
float time_kernel(K k, int grid, double* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, 0.999, 1e-3, out);  // warm
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, 0.999, 1e-3, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / 5;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int grid = cus * 8;  // 8 workgroups x 4 waves = 8 waves per SIMD
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * grid * 256));
  const float t_mfma = time_kernel(k_mfma, grid, out);
  const float t_valu = time_kernel(k_valu, grid, out);
  const float t_mixed = time_kernel(k_mixed, grid, out);
  CHECK(hipDeviceSynchronize());
  // per SIMD: waves = grid * 4 / (cus * 4) = 8
  const double waves_per_simd = grid * 4.0 / (cus * 4.0);
  const double mfma_per_simd = waves_per_simd * kIter * 4;
  const double valu_per_simd = waves_per_simd * kIter * 16;
  const double clk = 2.1e9;  // nominal under load; the ratios below do not depend on it
  std::printf("{\"cus\":%d,\"t_mfma_ms\":%.4f,\"t_valu_ms\":%.4f,\"t_mixed_ms\":%.4f,"
              "\"mfma_cycles_per_instr_at_2.1GHz\":%.2f,\"valu_cycles_per_instr_at_2.1GHz\":%.2f,"
              "\"mixed_over_max_of_halves\":%.3f}\n",
              cus, t_mfma, t_valu, t_mixed, t_mfma * 1e-3 * clk / mfma_per_simd,
              t_valu * 1e-3 * clk / valu_per_simd,
              t_mixed / (0.5 * (t_mfma > t_valu ? t_mfma : t_valu) + 1e-9));
  return 0;
}
