// Device integrand functors.
//
// Reference counterparts:
//   Pi4        — not in the reference; BASELINE.json's headline integrand 4/(1+x^2).
//   Sin        — riemann.cpp:37 / cintegrate.cu:68 (`sin(x)` on [0, pi]).
//   Poly       — BASELINE.json "random-init coefficients" synthetic integrand.
//   TrainVel   — riemann.cpp:103-116 vel_function (dead code there; live here).
//   Table      — cintegrate.cu:23-44 / 4main.c:249-269 linear interpolation of the
//                1801-sample velocity profile (ex4vel.h), staged in LDS instead of 3
//                global loads per sample, with the out-of-bounds read at t >= 1799
//                 fixed by clamping the segment index.
//
// Each functor exposes
//   point(x)           f(x) for one sample
//   tile<U>(x0, h)     sum_{u<U} f(x0 + u*h) — the hot loop, free to use a faster but
//                      still per-point-exact evaluation
//   kScale             constant factor folded into the final h*scale multiply
#pragma once

#include <hip/hip_runtime.h>

#include "miint/common.hpp"

namespace miint {

// ------------------------------------------------------------------ 4/(1+x^2), fp64
//
// Division is the whole cost of this integrand. The IEEE path (DivMode::kIeee) lets the
// compiler emit v_div_scale/v_rcp_f64/v_fma_f64 x4/v_div_fmas/v_div_fixup per point.
// The series path evaluates the same reciprocal per point from a per-tile seed:
//   s  ~= 1/d(x_mid)                 (v_rcp_f64 + one Newton step, once per U points)
//   e_u = 1 - d_u*s                  (exact residual via fma, |e_u| <= (U/2)*h*|f'/f| + eps)
//   1/d_u = s*(1 + e_u + e_u^2 + e_u^3/(1-e_u))
// |e_u| <= (U/2)*h (max of 2|x|/(1+x^2) is 1), so the dropped e^3 term is < 1e-17 relative
// whenever (U/2)*h <= 2e-6; the host dispatcher (series_ok()) falls back to kIeee otherwise.
// Every point is therefore still evaluated to fp64 accuracy; the per-point cost drops from ~10 VALU f64 ops to 5
// (x, d, e, and the two accumulations). Nothing is skipped: every sample x_u is formed and
// its reciprocal residual computed (tests check per-point agreement with IEEE division).
struct Pi4 {
  static constexpr double kScale = 4.0;

  __device__ __forceinline__ double point(double x) const { return 1.0 / fma(x, x, 1.0); }

  template <int U, DivMode M>
  __device__ __forceinline__ double tile(double x0, double h) const {
    if constexpr (M == DivMode::kIeee) {
      double acc = 0.0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double x = fma(static_cast<double>(u), h, x0);
        acc += 1.0 / fma(x, x, 1.0);
      }
      return acc;
    } else {
      const double xm = fma(0.5 * (U - 1), h, x0);
      const double dm = fma(xm, xm, 1.0);
      double s = __builtin_amdgcn_rcp(dm);
      s = fma(s, fma(-dm, s, 1.0), s);  // one Newton step: seed error ~1e-16 + |x-xm| term
      double t1a = 0.0, t1b = 0.0, t2 = 0.0;
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        const double xa = fma(static_cast<double>(u), h, x0);
        const double xb = fma(static_cast<double>(u + 1), h, x0);
        const double ea = fma(-fma(xa, xa, 1.0), s, 1.0);
        const double eb = fma(-fma(xb, xb, 1.0), s, 1.0);
        t1a += ea;
        t1b += eb;
        t2 = fma(ea, ea, t2);
        t2 = fma(eb, eb, t2);
      }
      // sum_u s*(1 + e_u + e_u^2): U*s + s*(sum e + sum e^2)
      return fma(s, (t1a + t1b) + t2, static_cast<double>(U) * s);
    }
  }
};

// ------------------------------------------------------------------ sin(x), fp64
struct Sin {
  static constexpr double kScale = 1.0;
  __device__ __forceinline__ double point(double x) const { return sin(x); }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    // ocml sin is ~40 VALU ops with its own range reduction; unrolling it fully blows the
    // register budget (256 VGPRs -> 1 wave/SIMD), two independent chains keep 8 waves/SIMD.
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll 1
    for (int u = 0; u < U; u += 2) {
      acc0 += sin(fma(static_cast<double>(u), h, x0));
      acc1 += sin(fma(static_cast<double>(u + 1), h, x0));
    }
    return acc0 + acc1;
  }
};

// ------------------------------------------------------------------ polynomial
struct Poly {
  static constexpr double kScale = 1.0;
  const double* c;  // points into the kernarg block (uniform -> SGPR loads)
  int n;
  __device__ __forceinline__ double point(double x) const {
    double r = 0.0;
    for (int k = n - 1; k >= 0; --k) r = fma(r, x, c[k]);
    return r;
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    double acc = 0.0;
#pragma unroll 4
    for (int u = 0; u < U; ++u) acc += point(fma(static_cast<double>(u), h, x0));
    return acc;
  }
};

// ------------------------------------------------------------------ analytic train velocity
// v(t) = (1 - cos(t/ts)) * vs   (riemann.cpp:108-111). Integral over [0,1800] is
// dis_function(1800) = vs*(1800 - ts*sin(1800/ts)) ~= 121999.99983.
struct TrainVel {
  double inv_ts, vs;
  static constexpr double kScale = 1.0;
  __device__ __forceinline__ double point(double t) const {
    return (1.0 - cos(t * inv_ts)) * vs;
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll 1
    for (int u = 0; u < U; u += 2) {
      acc0 += point(fma(static_cast<double>(u), h, x0));
      acc1 += point(fma(static_cast<double>(u + 1), h, x0));
    }
    return acc0 + acc1;
  }
};

// ------------------------------------------------------------------ velocity-profile table
// The 1801-sample table (14.4 KB) lives in LDS, loaded once per workgroup. Segment index is
// clamped to [0, nseg-1] so t == 1800 interpolates the last segment instead of reading
// past the end (the reference copies only 1800 of 1801 entries: cintegrate.cu:117,121).
struct Table {
  const double* lds;  // LDS copy of the table
  int nseg;           // number of segments = entries - 1
  static constexpr double kScale = 1.0;
  __device__ __forceinline__ double point(double t) const {
    int i = static_cast<int>(t);
    i = i < 0 ? 0 : (i >= nseg ? nseg - 1 : i);
    const double fr = t - static_cast<double>(i);
    const double v0 = lds[i];
    const double v1 = lds[i + 1];
    return fma(v1 - v0, fr, v0);
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int u = 0; u < U; u += 2) {
      acc0 += point(fma(static_cast<double>(u), h, x0));
      acc1 += point(fma(static_cast<double>(u + 1), h, x0));
    }
    return acc0 + acc1;
  }
};

}  // namespace miint
