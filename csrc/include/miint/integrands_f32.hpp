// Packed-fp32 integrand functors: sin, the analytic train velocity, the velocity table and
// polynomials (BASELINE.json config #4 "fp32 path ... error vs fp64" for the reference's own
// integrands: cintegrate.cu:47-72 sin, cintegrate.cu:74-98 the table interpolation).
//
// Same structure as Pi4F32 (riemann.hip) and the fp64 functors (integrands.hpp): the tile's
// anchor coordinate and its per-tile set-up (sin/cos seed, segment line, Taylor shift) are
// fp64, so sample coordinates never collapse (at N = 1e9 over [0, pi], h = 3.1e-9 is below
// ulp_f32(pi) = 2.4e-7: an fp32 coordinate a + i h would be the same float for ~77
// consecutive samples); every SAMPLE is then evaluated on its own in packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two samples per instruction, twice the work
// of an fp64 op per issue slot), accumulated in fp32 over one sub-tile or tile, and folded
// into the lane's fp64 sum. Nothing is merged across samples: the +k / -k samples of a pair
// are separate fmas and separate accumulations, exactly as in fp64.
//
// kIeee forms (the per-sample reference of each): fp64 coordinate per sample, fp32 math
// (ocml sinf / cosf, fp32 interpolation, fp32 Horner).
#pragma once

#include <hip/hip_runtime.h>

#include "miint/common.hpp"
#include "miint/integrands.hpp"

namespace miint {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ double fold(f32x2 a) {
  return static_cast<double>(a.x) + static_cast<double>(a.y);
}

// ------------------------------------------------------------------ angle series, fp32
// AngleSeries (integrands.hpp) with packed-fp32 samples: the per-tile sin/cos seed at the
// tile midpoint stays fp64 (tile_sincos), the 16-sample sub-tile centres are rotated from it
// in packed fp32 ((S_c, C_c) = (S c + C s, C c - S s), one pk_mul + one pk_fma), and each
// pair of offsets (k_j, k_{j+1}) is one pk_mul for the shared base term plus one pk_fma per
// sign for the samples: per 4 samples 1 pk_mul + 2 pk_fma + 2 pk_add (1.25 per sample).
template <int Subs>
struct AngleSeriesF32 {
  static constexpr int kPairs = 8;
  static constexpr int kSub = 2 * kPairs;
  static constexpr int kSubs = Subs;
  static constexpr int kSeriesTile = kSub * kSubs;
  static_assert(2 * kPairs + kSubs <= kSinTrig, "RiemannParams::trig layout");
  f32x2 ck[kPairs / 2], sk[kPairs / 2];  // (cos k_j d, cos k_{j+1} d), (sin ..., sin ...)
  float cc[kSubs / 2], sc[kSubs / 2];    // cos/sin(c0 d), c0 = 8, 24, ...

  // trig32: RiemannParams::trig rounded to fp32 on the host (kernel arguments -> SGPRs)
  __device__ __forceinline__ void init_trig(const float* trig) {
#pragma unroll
    for (int i = 0; i < kPairs / 2; ++i) {
      ck[i] = f32x2{trig[2 * i], trig[2 * i + 1]};
      sk[i] = f32x2{trig[kPairs + 2 * i], trig[kPairs + 2 * i + 1]};
    }
#pragma unroll
    for (int i = 0; i < kSubs / 2; ++i) {
      cc[i] = trig[2 * kPairs + 2 * i];
      sc[i] = trig[2 * kPairs + 2 * i + 1];
    }
  }
  // fp32 sum over a series tile anchored at theta_m of sin (COS = false) or cos (COS = true)
  template <bool COS>
  __device__ __forceinline__ f32x2 tile_sum(double theta_m) const {
    double Sd, Cd;
    tile_sincos(theta_m, Sd, Cd);
    const float S = static_cast<float>(Sd), C = static_cast<float>(Cd);
    f32x2 a = {0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < kSubs; ++q) {
      const int i = q < kSubs / 2 ? kSubs / 2 - 1 - q : q - kSubs / 2;
      const float c = cc[i], s = q < kSubs / 2 ? -sc[i] : sc[i];
      // (S_q, C_q) = (S c + C s, C c - S s)
      const f32x2 sq = pk_fma(f32x2{C, -S}, f32x2{s, s}, f32x2{S, C} * f32x2{c, c});
      const float base = COS ? sq.y : sq.x, side = COS ? -sq.x : sq.y;
      const f32x2 bb = {base, base}, sp = {side, side}, sn = {-side, -side};
#pragma unroll
      for (int j = 0; j < kPairs / 2; ++j) {
        const f32x2 u = bb * ck[j];
        a += pk_fma(sp, sk[j], u);  // theta_c + k delta, for k_{2j} and k_{2j+1}
        a += pk_fma(sn, sk[j], u);  // theta_c - k delta
        asm volatile("" : "+v"(a));  // keep program order (see Pi4)
      }
    }
    return a;
  }
};

// sin(x) in packed fp32 (cintegrate.cu:47-72's integrand, BASELINE #4).
struct SinF32 : TileDefaults<SinF32>, AngleSeriesF32<12> {
  static constexpr double kScale = 1.0;
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSeriesTile : 32;
  }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  __device__ __forceinline__ void init(const float* trig) { init_trig(trig); }
  __device__ __forceinline__ double point(double x) const {
    return static_cast<double>(sinf(static_cast<float>(x)));
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 1
    for (int u = 0; u < U; u += 2) {
      a0 += sinf(static_cast<float>(fma(static_cast<double>(u), h, x0)));
      a1 += sinf(static_cast<float>(fma(static_cast<double>(u + 1), h, x0)));
    }
    return static_cast<double>(a0) + static_cast<double>(a1);
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "angle series tiles are kSeriesTile samples");
      return acc + fold(tile_sum<false>(xa));
    } else {
      return acc + tile<U, M>(xa, h);
    }
  }
};

// (1 - cos(t/ts)) vs in packed fp32 (riemann.cpp:108-111): the tile value is
// vs (U - sum cos), the subtraction in fp64.
struct TrainVelF32 : TileDefaults<TrainVelF32>, AngleSeriesF32<8> {
  double inv_ts, vs;
  static constexpr double kScale = 1.0;
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSeriesTile : 32;
  }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  __device__ __forceinline__ double point(double t) const {
    return static_cast<double>((1.0f - cosf(static_cast<float>(t * inv_ts))) *
                               static_cast<float>(vs));
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    const float v = static_cast<float>(vs);
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 1
    for (int u = 0; u < U; u += 2) {
      a0 += (1.0f - cosf(static_cast<float>(fma(static_cast<double>(u), h, x0) * inv_ts))) * v;
      a1 += (1.0f - cosf(static_cast<float>(fma(static_cast<double>(u + 1), h, x0) * inv_ts))) * v;
    }
    return static_cast<double>(a0) + static_cast<double>(a1);
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double ta, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "angle series tiles are kSeriesTile samples");
      return fma(-vs, fold(tile_sum<true>(ta * inv_ts)), fma(vs, static_cast<double>(U), acc));
    } else {
      return acc + tile<U, M>(ta, h);
    }
  }
};

// ------------------------------------------------------------------ velocity table, fp32
// The segment-line tiles of Table (integrands.hpp), per sample in packed fp32: the tile's
// segment, its line (v_m, D = d h) and the kink are found in fp64 exactly as in fp64; each
// 32-sample sub-tile rounds its centre value once to fp32 and then forms every sample pair
// (v_c + k D, v_c - k D) with one pk_fma (+ pk_max / pk_fma for the kink) and accumulates it
// with one pk_add: 1 instruction per sample on a one-segment tile.
struct TableF32 : TileDefaults<TableF32> {
  const double* tab;  // the table (LDS copy for kIeee, global array for kSeries)
  int nseg;
  static constexpr double kScale = 1.0;
  static constexpr int kPairs = 16;
  static constexpr int kSub = 2 * kPairs;
  static constexpr int kSubs = 2;
  static constexpr int kSeriesTile = kSub * kSubs;
  double hspan = 0.5 * (kSeriesTile - 1);
  double inv_h = 0.0;
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSeriesTile : 32;
  }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  // Clamped in fp64 BEFORE the conversion: a double beyond the int range has no defined
  // static_cast<int> (the hardware saturates, the language does not promise it); NaN -> 0.
  __device__ __forceinline__ int segment(double t) const {
    return static_cast<int>(fmin(fmax(t, 0.0), static_cast<double>(nseg - 1)));
  }
  // fp64 coordinate and segment, fp32 interpolation
  __device__ __forceinline__ float pointf(double t) const {
    const int i = segment(t);
    const float fr = static_cast<float>(t - static_cast<double>(i));
    const float v0 = static_cast<float>(tab[i]);
    const float v1 = static_cast<float>(tab[i + 1]);
    return fmaf(v1 - v0, fr, v0);
  }
  __device__ __forceinline__ double point(double t) const {
    return static_cast<double>(pointf(t));
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 4
    for (int u = 0; u < U; u += 2) {
      a0 += pointf(fma(static_cast<double>(u), h, x0));
      a1 += pointf(fma(static_cast<double>(u + 1), h, x0));
    }
    return static_cast<double>(a0) + static_cast<double>(a1);
  }
  template <bool KINK>
  __device__ __forceinline__ double line_sum(double vm, double D, double dD, double kk) const {
    const float Df = static_cast<float>(D), dDf = static_cast<float>(dD);
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kSubs; ++q) {
      const double c0 = q == 0 ? -0.5 * kSub : 0.5 * kSub;
      const float vc = static_cast<float>(fma(c0, D, vm));
      const float r = static_cast<float>(c0 - kk);  // sub-tile centre relative to the knot
      f32x2 a = {0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < kPairs; ++j) {
        const float k = j + 0.5f;
        f32x2 g = pk_fma(f32x2{k, -k}, f32x2{Df, Df}, f32x2{vc, vc});  // (+k, -k) samples
        if constexpr (KINK) {
          const f32x2 over = __builtin_elementwise_max(f32x2{r + k, r - k}, f32x2{0.0f, 0.0f});
          g = pk_fma(over, f32x2{dDf, dDf}, g);
        }
        a += g;
        asm volatile("" : "+v"(a));
      }
      t += fold(a);
    }
    return t;
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xm, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "segment tiles are kSubs sub-tiles of kSub samples");
      const int lo = segment(fma(-hspan, h, xm)), hi = segment(fma(hspan, h, xm));
      if (lo == hi) {
        const double v0 = tab[lo], d = tab[lo + 1] - v0;
        return acc + line_sum<false>(fma(d, xm - static_cast<double>(lo), v0), d * h, 0.0, 0.0);
      }
      if (hi == lo + 1) {
        const double v0 = tab[lo], v1 = tab[lo + 1], v2 = tab[lo + 2];
        const double d0 = v1 - v0;
        return acc + line_sum<true>(fma(d0, xm - static_cast<double>(lo), v0), d0 * h,
                                    ((v2 - v1) - d0) * h,
                                    (static_cast<double>(lo + 1) - xm) * inv_h);
      }
      // coarse step (a tile spans several segments): per sample, rolled
      const double x0 = fma(-hspan, h, xm);
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 1
      for (int u = 0; u < U; u += 2) {
        s0 += pointf(fma(static_cast<double>(u), h, x0));
        s1 += pointf(fma(static_cast<double>(u + 1), h, x0));
      }
      return acc + (static_cast<double>(s0) + static_cast<double>(s1));
    } else {
      return acc + tile<U, M>(xm, h);
    }
  }
};

// ------------------------------------------------------------------ polynomial, fp32
// Poly's Taylor-pair tiles (integrands.hpp) in packed fp32: the shift to each 32-sample
// sub-tile centre is fp64 (b_m = h^m p^(m)(x_c) / m!, rounded once to fp32); two pairs
// (k_j, k_{j+1}) share one packed Horner of the even and odd parts at (k_j^2, k_{j+1}^2),
// then each sign is one pk_fma and one pk_add: NC - 1 + 4 packed ops per 4 samples.
template <int NC>
struct PolyF32 : TileDefaults<PolyF32<NC>> {
  static_assert(NC >= 2, "coefficient buckets are 4, 6, 7, 8 or 16 wide");
  static constexpr double kScale = 1.0;
  static constexpr int kPairs = 16;
  static constexpr int kSub = 2 * kPairs;
  static constexpr int kSubs = 2;
  static constexpr int kSeriesTile = kSub * kSubs;
  float c[NC];   // fp32 coefficients (kIeee Horner)
  double cs[NC]; // c_i h^i (series shift, fp64)
  double inv_h = 0.0;

  __device__ __forceinline__ void init(const double* coef, int n) {
#pragma unroll
    for (int k = 0; k < NC; ++k) c[k] = k < n ? static_cast<float>(coef[k]) : 0.0f;
  }
  __device__ __forceinline__ void init_series(const double* coef_h, int n, double h) {
#pragma unroll
    for (int k = 0; k < NC; ++k) cs[k] = k < n ? coef_h[k] : 0.0;
    inv_h = 1.0 / h;
  }
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSeriesTile : 32;
  }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  __device__ __forceinline__ float pointf(float x) const {
    float r = c[NC - 1];
#pragma unroll
    for (int k = NC - 2; k >= 0; --k) r = fmaf(r, x, c[k]);
    return r;
  }
  __device__ __forceinline__ double point(double x) const {
    return static_cast<double>(pointf(static_cast<float>(x)));
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll 4
    for (int u = 0; u < U; u += 2) {
      a0 += pointf(static_cast<float>(fma(static_cast<double>(u), h, x0)));
      a1 += pointf(static_cast<float>(fma(static_cast<double>(u + 1), h, x0)));
    }
    return static_cast<double>(a0) + static_cast<double>(a1);
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xm, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile && NC <= 8, "Taylor-pair tiles: NC <= 8, 64 samples");
      constexpr int ev = (NC - 1) & ~1, od = ((NC - 2) | 1);
      const double um = xm * inv_h;
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        // Taylor shift at the sub-tile centre (fp64), then the coefficients as packed pairs
        const double uc = um + (q == 0 ? -0.5 * kSub : 0.5 * kSub);
        double b[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) b[i] = cs[i];
#pragma unroll
        for (int m = 0; m < NC - 1; ++m)
#pragma unroll
          for (int i = NC - 2; i >= m; --i) b[i] = fma(b[i + 1], uc, b[i]);
        f32x2 bf[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) bf[i] = f32x2{static_cast<float>(b[i]), static_cast<float>(b[i])};
        f32x2 a = {0.0f, 0.0f};
#pragma unroll
        for (int j = 0; j < kPairs; j += 2) {
          const f32x2 k = {j + 0.5f, j + 1.5f};
          const f32x2 K = k * k;  // exact: (j + 1/2)^2 has at most 12 significant bits
          f32x2 E = bf[ev];
#pragma unroll
          for (int e = ev - 2; e >= 0; e -= 2) E = pk_fma(E, K, bf[e]);
          f32x2 O = bf[od];
#pragma unroll
          for (int o = od - 2; o >= 1; o -= 2) O = pk_fma(O, K, bf[o]);
          a += pk_fma(k, O, E);   // samples kSub/2 + j, kSub/2 + j + 1
          a += pk_fma(-k, O, E);  // samples kSub/2 - 1 - j, kSub/2 - 2 - j
          asm volatile("" : "+v"(a));
        }
        t += fold(a);
      }
      return acc + t;
    } else {
      return acc + tile<U, M>(xm, h);
    }
  }
};

}  // namespace miint
