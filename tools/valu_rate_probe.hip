// Microbenchmark: VALU issue cost per wave instruction on gfx950 for the forms the hot loops
// use — v_fma_f64, v_fma_f32, v_pk_fma_f32 (two fp32 lanes per op), v_pk_add_f32, and the
// reciprocal seeds v_rcp_f64 / v_rcp_f32 (alone and, for fp64, in the 1 + 6 fma mix) — with 8
// waves per SIMD and 8 independent chains per wave (throughput, not latency).
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate_probe.hip -o build/bin/valu_rate_probe
//   build/bin/valu_rate_probe            # one JSON line per form
//
// Question it answers: does the packed fp32 form the fp32 tiles use (integrands_f32.hpp)
// buy throughput on CDNA4, or does plain v_fma_f32 issue as fast per element?
// cycles/instr/SIMD = time x clock x SIMDs / (waves x instructions per wave), at the clock
// hipDeviceProp reports (an upper bound on the real clock under load, so the cycle counts
// are upper bounds too; the RATIOS between forms are what matters).
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

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 8192;
constexpr int kChains = 8;

template <class T>
__device__ __forceinline__ T fma_t(T a, T b, T c) {
  return __builtin_elementwise_fma(a, b, c);
}

// kind 0: f64 fma, 1: f32 fma, 2: packed f32 fma, 3: packed f32 add
template <int K>
__global__ __launch_bounds__(256) void k_rate(float a, float b, float* out) {
  if constexpr (K == 0) {
    double x[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = a + c;
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) x[c] = fma_t<double>(x[c], (double)a, (double)b);
      asm volatile("" ::: "memory");
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  } else if constexpr (K == 1) {
    float x[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = a + c;
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
      for (int c = 0; c < kChains; ++c)  // asm: left alone, hipcc packs the chains pairwise
        asm("v_fma_f32 %0, %1, %2, %3" : "=v"(x[c]) : "v"(x[c]), "v"(a), "v"(b));
      asm volatile("" ::: "memory");
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if constexpr (K == 4 || K == 6) {  // v_rcp_f64 chains; 6: one rcp + 6 fma each
    double x[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = a + c + 1.5;
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        x[c] = __builtin_amdgcn_rcp(x[c]);
        if constexpr (K == 6) {
#pragma unroll
          for (int f = 0; f < 6; ++f) x[c] = fma_t<double>(x[c], (double)a, (double)b);
        }
      }
      asm volatile("" ::: "memory");
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
  } else if constexpr (K == 5) {  // v_rcp_f32 chains
    float x[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = a + c + 1.5f;
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) x[c] = __builtin_amdgcn_rcpf(x[c]);
      asm volatile("" ::: "memory");
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    f32x2 x[kChains];
    const f32x2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = f32x2{a + c, b + c};
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        if constexpr (K == 2) x[c] = fma_t<f32x2>(x[c], va, vb);
        else x[c] = x[c] + vb;
      }
      asm volatile("" ::: "memory");
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c].x + x[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

template <int K>
int run(const char* name, int elems_per_instr, float* out, int grid, const hipDeviceProp_t& p) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_rate<K><<<grid, 256>>>(1.0000001f, 1e-7f, out);  // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    k_rate<K><<<grid, 256>>>(1.0000001f, 1e-7f, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double waves = grid * 4.0,
               instr = static_cast<double>(kIter) * kChains * (K == 6 ? 7 : 1);
  const double simds = p.multiProcessorCount * 4.0, clk = p.clockRate * 1e3;
  const double cyc = best * 1e-3 * clk * simds / (waves * instr);
  std::printf("{\"form\": \"%s\", \"ms\": %.4f, \"cycles_per_instr_per_simd\": %.3f, "
              "\"elements_per_instr\": %d, \"cycles_per_element_lane\": %.3f, \"clock_mhz\": %d}\n",
              name, best, cyc, elems_per_instr, cyc / elems_per_instr, p.clockRate / 1000);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount * 8;  // 8 workgroups of 4 waves per CU: 8 waves/SIMD
  float* out;
  CHECK(hipMalloc(&out, sizeof(float) * grid * 256));
  if (run<0>("v_fma_f64", 1, out, grid, p)) return 1;
  if (run<1>("v_fma_f32", 1, out, grid, p)) return 1;
  if (run<2>("v_pk_fma_f32", 2, out, grid, p)) return 1;
  if (run<3>("v_pk_add_f32", 2, out, grid, p)) return 1;
  if (run<4>("v_rcp_f64", 1, out, grid, p)) return 1;
  if (run<5>("v_rcp_f32", 1, out, grid, p)) return 1;
  // the narrow reciprocal's mix (integrands.hpp Pi4::recip_narrow): per instruction of 1 rcp + 6 fma
  if (run<6>("v_rcp_f64 + 6 v_fma_f64", 1, out, grid, p)) return 1;
  CHECK(hipFree(out));
  return 0;
}
