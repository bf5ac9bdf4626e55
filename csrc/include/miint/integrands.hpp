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

// Default tile hooks (CRTP). The lane loop calls
//   acc = f.tile_acc<U, M>(fma(i_anchor, h, a), h, acc)
// where i_anchor = first sample index of the tile + anchor<U, M>(): integrands whose hot
// path is centred on the tile (Pi4 series) ask for the midpoint directly, saving an fma.
template <class D>
struct TileDefaults {
  template <int U, DivMode M>
  __device__ static constexpr double anchor() { return 0.0; }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double x0, double h, double acc) const {
    return acc + static_cast<const D*>(this)->template tile<U, M>(x0, h);
  }
};

// ------------------------------------------------------------------ 4/(1+x^2), fp64
//
// Division is the whole cost of this integrand. The IEEE path (DivMode::kIeee) lets the
// compiler emit v_div_scale/v_rcp_f64/v_fma_f64 x4/v_div_fmas/v_div_fixup per point
// (~14 VALU f64 ops per sample with the coordinate and the accumulation).
//
// The series paths evaluate the same reciprocal per point from a per-tile seed:
//   s  ~= 1/d(x_m)                   (v_rcp_f64 + one Newton step, once per U points;
//                                     x_m = tile midpoint)
//   e_u = 1 - d(x_u)*s               (the point's exact residual)
//   1/d(x_u) = s*(1 + e_u + e_u^2 + e_u^3/(1-e_u))
// |e_u| <= (U/2)*h (max of 2|x|/(1+x^2) is 1), so the dropped e^3 term is < 1e-17 relative
// whenever (U/2)*h <= 2e-6; the host dispatcher (series_ok()) falls back to kIeee otherwise.
//
// kSeriesDirect forms x_u = x0 + u*h, d_u = 1 + x_u^2, e_u = 1 - d_u*s explicitly (5 ops).
// kSeries (default) evaluates the very same residual with the offset k = u - (U-1)/2 from
// the midpoint: since d(x_m + k h) = d_m + 2 x_m h k + h^2 k^2 exactly,
//   e_k = e_m + k*A + k^2*B,   A = -2 x_m h s,  B = -h^2 s,  e_m = 1 - d_m s,
// and the two samples at +-k share c_k = e_m + k^2 B:  e_{+-k} = c_k +- k A.
// That is 3 fma per PAIR of samples for the residuals plus 2 accumulations per sample
// (3.5 VALU ops per sample). It is not an approximation: the quadratic is exact, and it is
// more accurate than rounding x_u first. Every sample still gets its own residual and its
// own contribution; tests compare every point against IEEE division (<= 2 ulp).
struct Pi4 : TileDefaults<Pi4> {
  static constexpr double kScale = 4.0;
  static constexpr int kPairs = 16;  // supports tiles of up to 32 samples

  // Pair offsets k = j + 1/2, held in SGPRs for the whole kernel (see init()).
  // Every fma of the pair evaluation is then a 3-operand VOP3 v_fma_f64 with one SGPR
  // source; folded to literals instead, hipcc emits v_fmac_f64 + literal and has to copy the
  // shared c with a v_mov_b64 per pair (30 extra VALU per 32-sample tile, measured in the .s).
  double pk[kPairs];

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      double k = j + 0.5;
      asm volatile("" : "+s"(k));   // opaque -> stays an SGPR pair, never a literal
      pk[j] = k;
    }
  }

  __device__ __forceinline__ double point(double x) const { return 1.0 / fma(x, x, 1.0); }

  // Per-tile constants of the series reciprocal (also used by the validation kernel).
  struct Seed {
    double s, em, a, b;
  };
  __device__ __forceinline__ static Seed seed(double xm, double h) {
    const double dm = fma(xm, xm, 1.0);
    double s = __builtin_amdgcn_rcp(dm);
    s = fma(s, fma(-dm, s, 1.0), s);  // one Newton step
    return {s, fma(-dm, s, 1.0), (-2.0 * h) * xm * s, -(h * h) * s};
  }

  template <int U, DivMode M>
  __device__ __forceinline__ double tile(double x0, double h) const {
    static_assert(U % 2 == 0, "pair evaluation needs an even tile");
    if constexpr (M == DivMode::kIeee) {
      double acc = 0.0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double x = fma(static_cast<double>(u), h, x0);
        acc += 1.0 / fma(x, x, 1.0);
      }
      return acc;
    } else if constexpr (M == DivMode::kSeries) {
      return tile_acc<U, M>(fma(0.5 * (U - 1), h, x0), h, 0.0);
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

  // Hot path of the default kSeries mode: anchored at the tile midpoint x_m, one running
  // sum per side (e and e^2 folded into the same accumulator), and the tile's
  // s*(U + sum(e + e^2)) folded into the lane accumulator with a single fma.
  // Per 32-sample tile: 16 x 7 pair ops + ~12 seed/fold ops.
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      const Seed sd = seed(xa, h);
      double ta = 0.0, tb = 0.0;
      // c_j = e_m + k_j^2 B advanced by the exact integer step k_{j+1}^2 - k_j^2 = 2j + 2
      // (a literal operand of an in-place v_fmac: c_j is dead once e_{+-k_j} are formed),
      // so only k_j needs an SGPR pair: 32 SGPRs instead of 64 keeps the kernel at 7
      // resident workgroups per CU. The recurrence's rounding (|c| ~ 1e-8, 15 steps) stays
      // below 1e-22 absolute.
      double c = fma(0.25, sd.b, sd.em);
#pragma unroll
      for (int j = 0; j < U / 2; ++j) {
        static_assert(U / 2 <= kPairs, "tile larger than the pair table");
        const double k = pk[j];
        const double ep = fma(k, sd.a, c);   // sample u = U/2 + j
        const double en = fma(-k, sd.a, c);  // sample u = U/2 - 1 - j
        ta += ep;
        ta = fma(ep, ep, ta);
        tb += en;
        tb = fma(en, en, tb);
        if (j + 1 < U / 2) c = fma(static_cast<double>(2 * j + 2), sd.b, c);
      }
      return fma(sd.s, (ta + tb) + static_cast<double>(U), acc);
    } else {
      return acc + tile<U, M>(xa, h);
    }
  }
};

// ------------------------------------------------------------------ sin(x), fp64
struct Sin : TileDefaults<Sin> {
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
struct Poly : TileDefaults<Poly> {
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
struct TrainVel : TileDefaults<TrainVel> {
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
struct Table : TileDefaults<Table> {
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
