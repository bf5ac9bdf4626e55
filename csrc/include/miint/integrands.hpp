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
#include "miint/fast_trig.hpp"

namespace miint {

// Default tile hooks (CRTP). The lane loop calls
//   acc = f.tile_acc<U, M>(fma(i_anchor, h, a), h, acc)
// where i_anchor = first sample index of the tile + anchor<U, M>(): integrands whose hot
// path is centred on the tile (Pi4 series) ask for the midpoint directly, saving an fma.
template <class D>
struct TileDefaults {
  // Samples per lane tile (the grid-stride work unit) for division mode M.
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() { return 32; }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() { return 0.0; }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double x0, double h, double acc) const {
    return acc + static_cast<const D*>(this)->template tile<U, M>(x0, h);
  }
};

// ------------------------------------------------------------------ 4/(1+x^2), fp64
//
// Division is the whole cost of this integrand. The IEEE path (DivMode::kIeee) runs the
// library's division sequence per point, minus its range handling (recip_narrow: v_rcp_f64
// and 6 fma, bitwise IEEE; 10.4 VALU per sample with the coordinate and the accumulation,
// against 14.5 with v_div_scale/v_div_fmas/v_div_fixup).
//
// The series paths evaluate the same reciprocal per point from a per-tile seed:
//   s  ~= 1/d(x_m)                   (v_rcp_f64 once per tile; x_m = tile midpoint; the
//                                     kSeriesDirect seed adds one Newton step)
//   e_u = 1 - d(x_u)*s               (the point's exact residual)
//   1/d(x_u) = s*(1 + e_u + e_u^2 + e_u^3/(1-e_u))
// |e_u| <= |e_m| + (U/2)*h (max of 2|x|/(1+x^2) is 1), so the dropped e^3 term is < 1e-17
// relative whenever (U/2)*h <= 2e-6; the host dispatcher (series_ok(), kSeriesHalfSpan) falls
// back to kIeee otherwise.
//
// kSeriesDirect forms x_u = x0 + u*h, d_u = 1 + x_u^2, e_u = 1 - d_u*s explicitly (5 ops).
//
// kSeries (default) evaluates the very same residual from the offset k = u - (U-1)/2 to the
// midpoint: d(x_m + k h) = d_m + 2 x_m h k + h^2 k^2 exactly, so
//   e_k = e_m + k*A + k^2*B,   A = -2 x_m h s,  B = -h^2 s,  e_m = 1 - d_m s,
// and it folds the series into one square per sample:
//   1 + e + e^2 = 3/4 + g^2,   g = 1/2 + e,
// so a sample costs ONE accumulation, fma(g, g, t), instead of t += e; t = fma(e, e, t).
// The two samples at +-k of a sub-tile centre share c_k = 1/2 + e_c + k^2 B and get
// g_{+-k} = c_k +- k A. c_k is formed directly with one fma from an SGPR k^2 (no running
// recurrence: increments of ~1e-17 would be lost against ulp(1/2)). Per PAIR of samples:
// 1 fma for c_k, 2 for g, 2 accumulations = 2.5 VALU per sample.
// A 384-sample tile is 12 sub-tiles of 32 whose centres sit at c0 = -176, -144, ..., 144,
// 176 steps from x_m; re-expanding the exact quadratic there gives e_c = e_m + c0 A + c0^2 B
// and slope A' = A + 2 c0 B (3 fma per sub-tile, against ~10 for a fresh seed). The 16 pair
// constants k_j and k_j^2 - kMeanK2 sit in SGPRs and VGPRs, the centre tables in SGPRs.
// Measured (gfx950 .s, tools/isa_guard.py): 1007 VALU per 384-sample tile = 2.62 per sample
// (round 5; 192-sample tiles of 6: 508 = 2.65 — the per-seed work over twice the samples,
// 1.2 % less time for kSeries, 1.8 % for kSeriesExact, profiles/r5/tile384_ab.md; 128-sample
// tiles of 4: 342 = 2.67; 8 sub-tiles of 16: 354 per 128 = 2.77; 64-sample tiles with a
// Newton step: 183 per 64 = 2.86; the first form, t += e; t = fma(e, e, t) with one seed per
// 32 samples: 127 per 32 = 3.97).
//
// Accuracy: every sample still gets its own residual and its own contribution. Per point,
// g is rounded at ulp(1/2) scale: <= 5 ulp vs IEEE division anywhere. On the bench record's
// window (64 K samples from x = 0.125, N = 1e9; test_pi4_series_record_window): max 4 ulp,
// 82.5 % of points within 1 ulp (|d| <= 1), 98.0 % within 2 with 384-sample tiles (83.2 /
// 98.1 % with 192). (Round 1 quoted
// "92 % within 1": tools/ulp_probe.py then binned round(|d|), i.e. |d| < 1.5.) The sum agrees
// with the IEEE path to 1e-15 relative and |error| at N = 1e9 is unchanged (4.4e-16, mid).
struct Pi4 : TileDefaults<Pi4> {
  static constexpr double kScale = 4.0;
  static constexpr int kPairs = 16;                 // sample pairs per sub-tile
  static constexpr int kSub = 2 * kPairs;           // 32 samples per sub-tile
  // Sub-tiles per series tile: 12 (384 samples per seed; 6 sub-tiles ran 508 VALU per 192
  // samples, these 1007 per 384: 73.1 -> 71.8 us at N = 1e9 with series_exact). The longer
  // tile needs 192 h <= 2e-6 (kSeriesHalfSpan): N >= 9.6e7 on [0, 1].
  static constexpr int kSubs = 12;
  static constexpr int kSeriesTile = kSub * kSubs;  // 384 samples per seed
  // sum over a series tile's samples of k_u^2, k_u = u - (U-1)/2: 2 sum_{j<U/2} (j + 1/2)^2
  static constexpr double kSumK2 = (kSeriesTile / 2) * (kSeriesTile / 2 - 1) * (kSeriesTile - 1) / 3.0 +
                                   (kSeriesTile / 2) * (kSeriesTile / 2 - 1) + kSeriesTile / 4.0;
  static_assert(kSumK2 == 4718560.0, "sum of squared midpoint offsets of a 384-sample tile");

  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return (M == DivMode::kSeries || M == DivMode::kSeriesExact) ? kSeriesTile : 32;
  }

  // Constants held in registers for the whole kernel (see init()). Every fma of the pair
  // evaluation is then a 3-operand VOP3 v_fma_f64 with register sources; as literals, hipcc
  // has to use the 2-operand v_fmac_f64 and copy the shared operand with a v_mov_b64
  // (gfx9 VOP3 takes no literal). k_j and the centre constants live in SGPRs; the 16
  // k_j^2 - kMeanK2 would push the kernel past 96 allocated SGPRs (7 instead of 8 resident
  // workgroups per CU), so they sit in VGPRs instead (32 of the 64 a wave may hold at 8 waves
  // per SIMD), loaded once per kernel.
  // Mean of k_j^2 over a sub-tile's pairs: sum_j (j + 1/2)^2 / 16 = 1364/16.
  static constexpr double kMeanK2 = 85.25;
  static constexpr int kPk2Sgpr = 5;  // pk2[j < 5] in SGPRs: with the 6-sub-tile tables fills the 96
  double pk[kPairs];         // k_j = j + 1/2                          (SGPR)
  double pk2[kPairs];        // k_j^2 - kMeanK2                        (VGPR)
  double pc[kSubs / 2];      // |sub-tile centre offset| c0: 16, 48, 80 (SGPR)
  double pcm[kSubs / 2];     // c0 + kMeanK2 / c0                      (SGPR)
  double c15;                // 3/2 (e_m + 1/2 = 3/2 - d_m s in one fma)

  __device__ __forceinline__ static double opaque_s(double v) {
    asm volatile("" : "+s"(v));  // opaque -> stays an SGPR pair, never a literal
    return v;
  }
  __device__ __forceinline__ static double opaque_v(double v) {
    asm volatile("" : "+v"(v));  // opaque -> stays a VGPR pair
    return v;
  }
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      pk[j] = opaque_s(j + 0.5);
      const double k2 = (j + 0.5) * (j + 0.5) - kMeanK2;
      pk2[j] = j < kPk2Sgpr ? opaque_s(k2) : opaque_v(k2);
    }
#pragma unroll
    for (int i = 0; i < kSubs / 2; ++i) {
      const double c0 = kSub * (i + 0.5);
      pc[i] = opaque_s(c0);
      pcm[i] = opaque_s(c0 + kMeanK2 / c0);
    }
    c15 = opaque_s(1.5);
  }

  __device__ __forceinline__ double point(double x) const { return 1.0 / fma(x, x, 1.0); }

  // 1/d for 1 <= d <= 2^500, bitwise equal to IEEE division (the kIeee tiles). This is the
  // sequence hipcc -O3 emits for 1.0 / d on gfx950 —
  //   v_div_scale x2, v_rcp_f64, two Newton steps, q = 1 * r, rem = 1 - d q,
  //   v_div_fmas(rem, r, q), v_div_fixup
  // — without its range handling: for such d, v_div_scale returns its operands unscaled (no
  // denormal operand or quotient, exponent gap far below 768), so v_div_fmas is a plain fma,
  // and v_div_fixup returns the finite normal quotient unchanged. Every intermediate, and
  // the result, is therefore the library division's: 7 VALU (one v_rcp_f64) instead of 10.
  // The dispatcher runs Pi4Wide (the full division) when |x| can reach 2^249.
  __device__ __forceinline__ static double recip_narrow(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    r = fma(r, fma(-d, r, 1.0), r);
    return fma(fma(-d, r, 1.0), r, r);
  }

  // Per-tile seed for kSeriesDirect (also the reciprocal seed of kSeries).
  struct Seed {
    double s, em, a, b;
  };
  __device__ __forceinline__ static Seed seed(double xm, double h) {
    const double dm = fma(xm, xm, 1.0);
    double s = __builtin_amdgcn_rcp(dm);
    s = fma(s, fma(-dm, s, 1.0), s);  // one Newton step
    return {s, fma(-dm, s, 1.0), (-2.0 * h) * xm * s, -(h * h) * s};
  }
  // kSeries seed: the raw v_rcp_f64 — no Newton step: the series is exact for any seed whose
  // residual keeps e^3 negligible (e_m is formed from the s actually used), and the per-point
  // error distribution measured with and without the step is the same (max 5 ulp) — with
  // eh = 1/2 + e_m rounded once (3/2 - d_m s).
  __device__ __forceinline__ Seed seed_half(double xm, double h) const {
    const double dm = fma(xm, xm, 1.0);
    const double s = __builtin_amdgcn_rcp(dm);
    return {s, fma(-dm, s, c15), (-2.0 * h) * xm * s, -(h * h) * s};
  }
  // Sub-tile q's centre offset c0 (in steps from x_m), c0 + kMeanK2/c0 and 2 c0, from the
  // SGPR table (negative side by the free source-negate modifier).
  __device__ __forceinline__ static double side(const double* t, int q) {
    return q < kSubs / 2 ? -t[kSubs / 2 - 1 - q] : t[q - kSubs / 2];
  }
  // g at sub-tile centre, carrying the sub-tile's mean k^2 B:
  //   1/2 + e_m + c0 A + (c0^2 + kMeanK2) B = fma(c0, fma(c0 + kMeanK2/c0, B, A), 1/2 + e_m).
  // Each pair then adds only (k^2 - kMeanK2) B, which sums to zero over the sub-tile: when
  // that term is below half an ulp of 1/2 (h ~ 1e-9) and fma(., ., eh) drops it, the dropped
  // amounts cancel instead of biasing every sample the same way (B < 0), which they did
  // (+0.2..0.4 ulp mean per point) with plain k^2.
  __device__ __forceinline__ double centre_g(const Seed& sd, int q) const {
    return fma(side(pc, q), fma(side(pcm, q), sd.b, sd.a), sd.em);
  }
  // slope at the centre, A + 2 c0 B, from b2 = 2 B (formed once per tile: a 2 c0 table would
  // push the kernel past 96 allocated SGPRs, i.e. 7 instead of 8 resident workgroups per CU)
  __device__ __forceinline__ double centre_slope(const Seed& sd, double b2, int q) const {
    return fma(side(pc, q), b2, sd.a);
  }

  template <int U, DivMode M>
  __device__ __forceinline__ double tile(double x0, double h) const {
    static_assert(U % 2 == 0, "pair evaluation needs an even tile");
    static_assert(M != DivMode::kSeries, "kSeries runs through tile_acc");
    if constexpr (M == DivMode::kIeee) {
      double acc = 0.0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double x = fma(static_cast<double>(u), h, x0);
        acc += recip_narrow(fma(x, x, 1.0));
      }
      return acc;
    } else {
      const Seed sd = seed(fma(0.5 * (U - 1), h, x0), h);
      double t1a = 0.0, t1b = 0.0, t2 = 0.0;
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        const double xa = fma(static_cast<double>(u), h, x0);
        const double xb = fma(static_cast<double>(u + 1), h, x0);
        const double ea = fma(-fma(xa, xa, 1.0), sd.s, 1.0);
        const double eb = fma(-fma(xb, xb, 1.0), sd.s, 1.0);
        t1a += ea;
        t1b += eb;
        t2 = fma(ea, ea, t2);
        t2 = fma(eb, eb, t2);
      }
      // sum_u s*(1 + e_u + e_u^2): U*s + s*(sum e + sum e^2)
      return fma(sd.s, (t1a + t1b) + t2, static_cast<double>(U) * sd.s);
    }
  }

  // kSeries tiles are anchored at their midpoint; the lane loop passes x_m directly.
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return (M == DivMode::kSeries || M == DivMode::kSeriesExact) ? 0.5 * (U - 1) : 0.0;
  }

  // kSeriesExact: the same seed, centres and per-sample residuals as kSeries, without the
  // 1/2 offset — e_c = e_m + c0 A + (c0^2 + kMeanK2) B, e_{+-k} = e_c + (k^2 - kMeanK2) B
  // +- k A' — and every sample's value is s (1 + e + e^2) at e's own precision (|e| <= 2e-6:
  // its rounding is ~1e-22 absolute), rounded once, where kSeries's g = 1/2 + e rounds every
  // sample at ulp(1/2) (up to 5 ulp from IEEE division).
  // Cost (round 5): each sample forms its own residual e+-k and adds its
  // own e^2 with one fma, exactly as kSeries forms g+-k and adds g^2 (whose square carries
  // the linear term g^2 = 1/4 + e + e^2). The residuals' LINEAR terms are not added sample by
  // sample: over the tile, e_u = e_m + k_u A + k_u^2 B with offsets k_u = u - (U-1)/2
  // symmetric about the midpoint, so sum_u e_u = U e_m + B sum_u k_u^2 exactly (the A terms
  // cancel) — one fma per tile, exact where per-sample adds would round. Per pair: c, e+, e-,
  // two fma = 2.5 VALU per sample, kSeries's count (the first form, f = fma(e, e, e) and
  // t += f per sample, was 3.5: +37 % time).
  // The seed's residual e_m = 1 - (1 + x_m^2) s is formed from the exact d_m (x_m s split
  // into q + qe by an fma): from the rounded d_m = fma(x_m, x_m, 1) it carried d_m's
  // rounding (up to ulp(1)/2 relative) into every sample of the tile — the 1.49-ulp maximum
  // near x = 0 of round 4 (profiles/r4/accuracy_ab.md).
  __device__ __forceinline__ Seed seed_exact(double xm, double h) const {
    const double dm = fma(xm, xm, 1.0);
    const double s = __builtin_amdgcn_rcp(dm);
    const double q = xm * s;
    const double qe = fma(xm, s, -q);  // xm s = q + qe exactly
    // 1 - s is exact for s in [1/2, 2] (d in [1/2, 2]: x in [0, 1]); elsewhere the rounding
    // is no worse than 1 - d_m s's
    const double em = fma(-xm, qe, fma(-xm, q, 1.0 - s));
    return {s, em, (-2.0 * h) * xm * s, -(h * h) * s};
  }

  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "series tiles are kSubs sub-tiles of kSub samples");
      const Seed sd = seed_half(xa, h);
      const double b2 = 2.0 * sd.b;
      // One running sum for the whole tile, started at the tile's U * 3/4. Its rounding
      // (ulp(64) ~ 1.4e-14) is far below the lane accumulator's it is folded into (~1.5e3
      // after 30 tiles, ulp 2.3e-13); a single chain is fine at 8 waves per SIMD.
      double t = 0.75 * U;
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        const double eh = centre_g(sd, q);     // 1/2 + e at the centre (+ mean k^2 B)
        const double a = centre_slope(sd, b2, q);  // slope there
#pragma unroll
        for (int j = 0; j < kPairs; ++j) {
          const double c = fma(pk2[j], sd.b, eh);
          const double gp = fma(pk[j], a, c);   // sample kSub/2 + j of the sub-tile
          const double gn = fma(-pk[j], a, c);  // sample kSub/2 - 1 - j
          t = fma(gp, gp, t);
          t = fma(gn, gn, t);
          // Keep program order (empty asm, no instructions): left free, the scheduler
          // hoists and interleaves the sub-tiles' independent chains and, with all of
          // them live, trades the 3-operand v_fma_f64 for v_fmac_f64 + v_mov_b64 copies.
          asm volatile("" : "+v"(t));
        }
      }
      return fma(sd.s, t, acc);
    } else if constexpr (M == DivMode::kSeriesExact) {
      static_assert(U == kSeriesTile, "series tiles are kSubs sub-tiles of kSub samples");
      const Seed sd = seed_exact(xa, h);
      const double b2 = 2.0 * sd.b;
      // sum_u e_u (U e_m + B sum k^2), then every sample's e^2 on top (|t| <= ~1e-12)
      double t = fma(kSumK2, sd.b, static_cast<double>(U) * sd.em);
#if MIINT_PI4_PIPE
      // Software-pipelined by one pair: pair p+1's residuals are formed between pair p's two
      // accumulations, so no instruction waits on the one issued just before it (at one
      // wave per SIMD nothing else would fill that gap). Same operations, same order of the
      // t accumulations: bitwise the plain loop's value. The empty asm statements pin the
      // order (each takes the value just produced and the operand of the next instruction).
      constexpr int kN = kSubs * kPairs;
      double ec = centre_g(sd, 0), a = centre_slope(sd, b2, 0);
      double c = fma(pk2[0], sd.b, ec);
      double en = fma(-pk[0], a, c);
      double ep = fma(pk[0], a, c);
#pragma unroll
      for (int p = 1; p < kN; ++p) {
        const int q = p / kPairs, j = p % kPairs;
        if (j == 0) {
          ec = centre_g(sd, q);
          a = centre_slope(sd, b2, q);
        }
        double c2 = fma(pk2[j], sd.b, ec);
        asm volatile("" : "+v"(c2), "+v"(t));
        t = fma(ep, ep, t);
        asm volatile("" : "+v"(t), "+v"(c2));
        double en2 = fma(-pk[j], a, c2);
        asm volatile("" : "+v"(en2), "+v"(t));
        t = fma(en, en, t);
        asm volatile("" : "+v"(t), "+v"(c2));
        double ep2 = fma(pk[j], a, c2);
        asm volatile("" : "+v"(ep2), "+v"(ec));
        en = en2;
        ep = ep2;
      }
      t = fma(ep, ep, t);
      t = fma(en, en, t);
#else
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        const double ec = centre_g(sd, q);         // e at the centre (+ mean k^2 B)
        const double a = centre_slope(sd, b2, q);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) {
          const double c = fma(pk2[j], sd.b, ec);
          const double ep = fma(pk[j], a, c);   // sample kSub/2 + j's residual
          const double en = fma(-pk[j], a, c);  // sample kSub/2 - 1 - j's
          t = fma(ep, ep, t);
          t = fma(en, en, t);
          // program order, as kSeries. (One chain even at 1 wave per SIMD: two running sums,
          // e+ and e- apart, ran 4-5 % slower at G = 1 and at the 1/4 and 1/8 shares,
          // profiles/r6/batch_tail.md.)
          asm volatile("" : "+v"(t));
        }
      }
#endif
      // U samples of s (1 + e + e^2): s U + s (sum e + sum e^2)
      return fma(sd.s, t, fma(sd.s, static_cast<double>(U), acc));
    } else {
      return acc + tile<U, M>(xa, h);
    }
  }

  // kSeriesExact value of sample u of a full tile (validation kernel): s + s (e + e^2), one
  // rounding, from the same seed, centre and residual e as the tile. The tile itself does
  // not form this per-sample value: it adds the residuals' linear terms once per tile
  // (s U + s (U e_m + B sum k^2 + sum e^2)), so the two differ by roundings only; over one
  // full tile they agree to a few ulp of the tile sum
  // (test_pi4_series_exact_point_kernel_sums_to_the_tile).
  __device__ __forceinline__ double series_exact_point(double xm, double h, int u) const {
    const Seed sd = seed_exact(xm, h);
    const double b2 = 2.0 * sd.b;
    const int q = u / kSub, w = u % kSub;
    const double ec = centre_g(sd, q);
    const double a = centre_slope(sd, b2, q);
    const int j = w >= kSub / 2 ? w - kSub / 2 : kSub / 2 - 1 - w;
    const double c = fma(pk2[j], sd.b, ec);
    const double e = w >= kSub / 2 ? fma(pk[j], a, c) : fma(-pk[j], a, c);
    return fma(sd.s, fma(e, e, e), sd.s);
  }

  // Series value of sample u of a full tile, by exactly the operations tile_acc applies to
  // it (validation kernel): s * (3/4 + g_u^2).
  __device__ __forceinline__ double series_point(double xm, double h, int u) const {
    const Seed sd = seed_half(xm, h);
    const double b2 = 2.0 * sd.b;
    const int q = u / kSub, w = u % kSub;
    const double eh = centre_g(sd, q);
    const double a = centre_slope(sd, b2, q);
    const int j = w >= kSub / 2 ? w - kSub / 2 : kSub / 2 - 1 - w;
    const double c = fma(pk2[j], sd.b, eh);
    const double g = w >= kSub / 2 ? fma(pk[j], a, c) : fma(-pk[j], a, c);
    return sd.s * fma(g, g, 0.75);
  }
};

// 4/(1+x^2) by the library's full IEEE division, for kIeee launches whose coordinates can
// reach |x| >= 2^249 (1 + x^2 beyond Pi4::recip_narrow's range: the quotient nears the
// denormals, 1 + x^2 may overflow). The dispatcher picks it from the launch's end points.
struct Pi4Wide : TileDefaults<Pi4Wide> {
  static constexpr double kScale = 4.0;
  __device__ __forceinline__ double point(double x) const { return 1.0 / fma(x, x, 1.0); }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile(double x0, double h) const {
    static_assert(M == DivMode::kIeee, "wide-domain Pi4 runs IEEE division only");
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += point(fma(static_cast<double>(u), h, x0));
    return acc;
  }
};
// Largest |x| for which every 1 + x^2 stays inside Pi4::recip_narrow's range.
constexpr double kPi4NarrowMaxX = 0x1p249;

// ------------------------------------------------------------------ tile seed: sin and cos
// sin and cos of a tile midpoint angle (|theta| up to ~1e5; the integrands use [0, 2 pi]):
// n = rint(theta 2/pi), r = theta - n pi/2 by a two-part Cody-Waite reduction (pi/2 = hi + lo,
// hi with 33 significant bits, so n hi is exact and both fma steps round only at ulp(r)),
// then the fdlibm kernel polynomials on [-pi/4, pi/4] (sin: odd degree 13; cos: even degree
// 14 with the 1 - z/2 split that keeps it within 1 ulp), and the quadrant's swap and signs.
// ~40 VALU against ~110 for ocml sincos (general range reduction with a Payne-Hanek path),
// which was ~0.9 VALU per sample of a 128-sample angle-addition tile.
__device__ __forceinline__ void tile_sincos(double th, double& S, double& C) {
  constexpr double kTwoOverPi = 6.36619772367581382433e-01;
  constexpr double kPio2Hi = 1.57079632673412561417e+00;  // 0x1.921fb544p+0
  constexpr double kPio2Lo = 6.07710050650619224932e-11;  // pi/2 - kPio2Hi
  const double n = rint(th * kTwoOverPi);
  const double r = fma(-n, kPio2Lo, fma(-n, kPio2Hi, th));
  const int q = static_cast<int>(n);
  const double z = r * r, w = z * z;
  // sin r = r + r z (S1 + z (S2 + ... + z S6))
  const double s26 = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10,
                                                -2.50507602534068634195e-08),
                                           2.75573137070700676789e-06),
                                      -1.98412698298579493134e-04),
                         8.33333333332248946124e-03);
  const double sr = fma(r * z, fma(z, s26, -1.66666666666666324348e-01), r);
  // cos r = (1 - z/2) + (((1 - (1 - z/2)) - z/2) + z (z (C1 + z C2 + z^2 C3) + z^4 (C4 + ...)))
  const double c13 = fma(z, fma(z, 2.48015872894767294178e-05, -1.38888888888741095749e-03),
                         4.16666666666666019037e-02);
  const double c46 = fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                         -2.75573143513906633035e-07);
  const double rc = fma(w * w, c46, z * c13);
  const double hz = 0.5 * z, cw = 1.0 - hz;
  const double cc = cw + (((1.0 - cw) - hz) + z * rc);
  const bool swap = (q & 1) != 0;
  const double a = swap ? cc : sr, b = swap ? sr : cc;
  S = (q & 2) ? -a : a;
  C = ((q + 1) & 2) ? -b : b;
}

// ------------------------------------------------------------------ sin / cos by angle addition
// Shared series path of Sin and TrainVel (both evaluate sin or cos of theta = w x):
// one sin/cos pair per tile at the midpoint theta_m (tile_sincos), re-centred to Subs
// 16-sample sub-tiles (centres theta_m + c0 delta, c0 = +-8, +-24, +-40, ...;
// delta = w h), then every sample by the exact angle-addition formula
//   sin(theta_c +- k delta) = S_c cos(k delta) +- C_c sin(k delta)
//   cos(theta_c +- k delta) = C_c cos(k delta) -+ S_c sin(k delta)
// with cos/sin(k delta) for the 8 pair offsets k = j + 1/2 and for the centres computed once
// per launch on the host in long double (RiemannParams::trig, kernel arguments -> SGPRs).
// Per pair: 1 mul + 2 fma for the two samples + 2 accumulations (2.5 VALU per sample); the
// seed (~40 VALU) and the 4-op re-centring per sub-tile add the rest: ~388 VALU per tile at
// Subs = 8 (TrainVel, 128 samples), ~580 at Subs = 12 (Sin, 192 samples); measured per
// sample: 2.98 (Sin) and 3.13 (TrainVel) VALU (profiles/r2/fp32_counters.md, fp64 rows).
// Every centre comes straight from the tile midpoint (one rounding), so the per-point error
// does not grow with the tile. No truncation (valid for any h).
// Subs sub-tiles per seed: Sin runs 12 (192-sample tiles, 1.20e13 -> 1.24e13 subint/s over
// 8), TrainVel keeps 8 (12 measured 1.18e13 -> 1.15e13). The host fills the centre table for
// the largest Subs; a smaller Subs reads its prefix (the same c0 = 8, 24, ... values).
template <int Subs>
struct AngleSeries {
  static constexpr int kPairs = 8;
  static constexpr int kSub = 2 * kPairs;
  static constexpr int kSubs = Subs;
  static constexpr int kSeriesTile = kSub * kSubs;
  static_assert(2 * kPairs + kSubs <= kSinTrig, "RiemannParams::trig layout");
  double ck[kPairs], sk[kPairs];       // cos(k_j delta), sin(k_j delta)
  double cc[kSubs / 2], sc[kSubs / 2];  // cos/sin(c0 delta), c0 = 8, 24, ..., 88

  __device__ __forceinline__ void init_trig(const double* trig) {
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      ck[j] = trig[j];
      sk[j] = trig[kPairs + j];
    }
#pragma unroll
    for (int i = 0; i < kSubs / 2; ++i) {
      cc[i] = trig[2 * kPairs + 2 * i];
      sc[i] = trig[2 * kPairs + 2 * i + 1];
    }
  }
  // sin and cos at the centre of sub-tile q (centre offsets -88, -72, ..., 72, 88 steps)
  __device__ __forceinline__ void centre(double S, double C, int q, double& Sq,
                                         double& Cq) const {
    const int i = q < kSubs / 2 ? kSubs / 2 - 1 - q : q - kSubs / 2;
    const double c = cc[i], s = q < kSubs / 2 ? -sc[i] : sc[i];
    Sq = fma(C, s, S * c);
    Cq = fma(-S, s, C * c);
  }
  // sum over a series tile anchored at theta_m of sin (COS = false) or cos (COS = true)
  template <bool COS>
  __device__ __forceinline__ double tile_sum(double theta_m) const {
    double S, C;
    tile_sincos(theta_m, S, C);
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kSubs; ++q) {
      double Sq, Cq;
      centre(S, C, q, Sq, Cq);
      const double base = COS ? Cq : Sq, side = COS ? -Sq : Cq;
#pragma unroll
      for (int j = 0; j < kPairs; ++j) {
        const double u = base * ck[j];
        t += fma(side, sk[j], u);   // theta_c + k_j delta
        t += fma(-side, sk[j], u);  // theta_c - k_j delta
        asm volatile("" : "+v"(t));  // keep program order (see Pi4)
      }
    }
    return t;
  }
  // sample u of a full series tile, by exactly tile_sum's operations (validation kernel)
  template <bool COS>
  __device__ __forceinline__ double point_of(double theta_m, int u) const {
    double S, C, Sq, Cq;
    tile_sincos(theta_m, S, C);
    const int q = u / kSub, w = u % kSub;
    centre(S, C, q, Sq, Cq);
    const double base = COS ? Cq : Sq, side = COS ? -Sq : Cq;
    const int j = w >= kSub / 2 ? w - kSub / 2 : kSub / 2 - 1 - w;
    const double v = base * ck[j];
    return w >= kSub / 2 ? fma(side, sk[j], v) : fma(-side, sk[j], v);
  }
};

// ------------------------------------------------------------------ per-sample trig tiles
// kIeee tiles of Sin and TrainVel: every sample's own sin/cos by fast_trig.hpp (tile-shared
// quadrant and Cody-Waite products, fdlibm kernels with the reduction tail), ocml per sample
// for the tiles it declines. ANGLE maps the sample coordinate to the angle (identity for
// sin, t / ts for the train); SHIFT 0 sums sin, 1 sums cos. Returns the signed sum over the
// tile's U samples x0 + u h.
template <int U, int SHIFT, class ANGLE, class LIB>
__device__ __forceinline__ double trig_tile_sum(double x0, double h, const ANGLE& angle,
                                                const LIB& lib) {
  TrigTile q;
  if (trig_tile(angle(x0), angle(fma(static_cast<double>(U - 1), h, x0)), SHIFT, q)) {
    double a0 = 0.0, a1 = 0.0;
    if (q.use_cos) {
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        a0 += trig_sample<true>(angle(fma(static_cast<double>(u), h, x0)), q);
        a1 += trig_sample<true>(angle(fma(static_cast<double>(u + 1), h, x0)), q);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        a0 += trig_sample<false>(angle(fma(static_cast<double>(u), h, x0)), q);
        a1 += trig_sample<false>(angle(fma(static_cast<double>(u + 1), h, x0)), q);
      }
    }
    const double t = a0 + a1;
    return q.neg ? -t : t;
  }
  double acc0 = 0.0, acc1 = 0.0;  // library per sample (two chains keep 8 waves/SIMD)
#pragma unroll 1
  for (int u = 0; u < U; u += 2) {
    acc0 += lib(angle(fma(static_cast<double>(u), h, x0)));
    acc1 += lib(angle(fma(static_cast<double>(u + 1), h, x0)));
  }
  return acc0 + acc1;
}
// Sample u of a kIeee trig tile by exactly trig_tile_sum's operations (validation kernel).
template <int U, int SHIFT, class ANGLE, class LIB>
__device__ __forceinline__ double trig_tile_point(double x0, double h, int u, const ANGLE& angle,
                                                  const LIB& lib) {
  TrigTile q;
  const double th = angle(fma(static_cast<double>(u), h, x0));
  if (!trig_tile(angle(x0), angle(fma(static_cast<double>(U - 1), h, x0)), SHIFT, q))
    return lib(th);
  const double v = q.use_cos ? trig_sample<true>(th, q) : trig_sample<false>(th, q);
  return q.neg ? -v : v;
}
struct IdentityAngle {
  __device__ __forceinline__ double operator()(double x) const { return x; }
};
struct ScaledAngle {
  double k;
  __device__ __forceinline__ double operator()(double x) const { return x * k; }
};
struct OcmlSin {
  __device__ __forceinline__ double operator()(double x) const { return sin(x); }
};
struct OcmlCos {
  __device__ __forceinline__ double operator()(double x) const { return cos(x); }
};

// ------------------------------------------------------------------ sin(x), fp64
// kIeee: every sample's own sin (trig_tile_sum: fast_trig.hpp per sample, ocml for tiles
// it declines); SinLib keeps ocml sin for every sample (~56 VALU, with its range reduction:
// the validation reference).
// kSeries (default): AngleSeries<12> with w = 1 (192-sample tiles). Per point: absolute
// error vs ocml sin <= 7.2e-16 measured (tests allow 4 ulp(1)); the sum agrees with the kIeee
// path to 2e-15 relative. N = 1e9 on [0, pi]: 81.2 us per integration (1.23e13 subint/s,
// profiles/r2/bench_fp32_all.jsonl) vs 1.53 ms for ocml sin per sample.
struct Sin : TileDefaults<Sin>, AngleSeries<12> {
  static constexpr double kScale = 1.0;
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSeriesTile : 32;
  }
  template <int U, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (U - 1) : 0.0;
  }
  __device__ __forceinline__ void init(const double* trig) { init_trig(trig); }
  __device__ __forceinline__ double point(double x) const { return sin(x); }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "angle series tiles are kSeriesTile samples");
      return acc + tile_sum<false>(xa);
    } else {
      return acc + tile<U, M>(xa, h);
    }
  }
  __device__ __forceinline__ double series_point(double xm, int u) const {
    return point_of<false>(xm, u);
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    return trig_tile_sum<U, 0>(x0, h, IdentityAngle{}, OcmlSin{});
  }
  template <int U>
  __device__ __forceinline__ double ieee_point(double x0, double h, int u) const {
    return trig_tile_point<U, 0>(x0, h, u, IdentityAngle{}, OcmlSin{});
  }
};
// ocml sin for every sample (validation reference of the kIeee tile; set_trig_library).
struct SinLib : Sin {
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
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    static_assert(M != DivMode::kSeries, "SinLib is the kIeee reference");
    return acc + tile<U, M>(xa, h);
  }
  template <int U>
  __device__ __forceinline__ double ieee_point(double x0, double h, int u) const {
    return sin(fma(static_cast<double>(u), h, x0));
  }
};

// ------------------------------------------------------------------ polynomial
// kIeee: Horner over a compile-time bucket of NC coefficients (4, 8 or 16), zero-padded at
// the top (leading zeros keep r == 0 exactly), per sample: NC - 1 fma plus the coordinate
// and the accumulation. The coefficients are copied into the functor once per kernel
// (uniform -> SGPRs): a runtime-length loop over a kernarg pointer reloaded every
// coefficient of every sample through the scalar cache (1.19 ms per 1e9 samples at degree 6
// vs this form's NC fma per sample).
//
// kSeries (NC <= 8): Taylor-pair tiles. A 64-sample tile is two 32-sample sub-tiles; at a
// sub-tile centre x_c the polynomial in the step offset k is q(k) = p(x_c + k h) =
// sum_m b_m k^m with b_m = h^m p^(m)(x_c)/m!, obtained by the repeated-Horner Taylor shift
// of p~(u) = sum_i (c_i h^i) u^i at u_c = x_c / h (NC (NC - 1) / 2 fma; the host supplies
// c_i h^i, so the b_m come out already scaled). The two samples at +-k share the even and
// odd parts E(k^2) = b_0 + k^2 b_2 + ..., O(k^2) = b_1 + k^2 b_3 + ...: p(x_c +- k h) =
// E +- k O, each sample its own fma and accumulation. Degree 6/7: 10 VALU per pair plus the
// shift, ~5.9 per sample against ~10 for Horner; exact algebra, valid for any h.
template <int NC>
struct Poly : TileDefaults<Poly<NC>> {
  static constexpr double kScale = 1.0;
  static constexpr int kPairs = 16;                 // sample pairs per sub-tile
  static constexpr int kSub = 2 * kPairs;           // 32 samples per sub-tile
  static constexpr int kSubs = 2;                   // sub-tile centres at -16, +16 steps
  static constexpr int kSeriesTile = kSub * kSubs;  // 64 samples per tile
  double c[NC];
  // series path only (init_series)
  double cs[NC];       // c_i h^i
  double pk[kPairs];   // k_j = j + 1/2 (SGPR; k_j^2 is formed from it: a k^2 table spilled)
  double c16;          // sub-tile centre offset
  double inv_h;

  __device__ __forceinline__ void init(const double* coef, int n) {
#pragma unroll
    for (int k = 0; k < NC; ++k) c[k] = k < n ? coef[k] : 0.0;
  }
  __device__ __forceinline__ void init_series(const double* coef_h, int n, double h) {
#pragma unroll
    for (int k = 0; k < NC; ++k) cs[k] = k < n ? coef_h[k] : 0.0;
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      double v = j + 0.5;
      asm volatile("" : "+s"(v));
      pk[j] = v;
    }
    double v = 0.5 * kSub;
    asm volatile("" : "+s"(v));
    c16 = v;
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
  __device__ __forceinline__ double point(double x) const {
    double r = c[NC - 1];
#pragma unroll
    for (int k = NC - 2; k >= 0; --k) r = fma(r, x, c[k]);
    return r;
  }
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    double acc = 0.0;
#pragma unroll 4
    for (int u = 0; u < U; ++u) acc += point(fma(static_cast<double>(u), h, x0));
    return acc;
  }
  // Taylor coefficients b_0..b_{NC-1} (scaled by h^m) at u_c = x_c / h.
  __device__ __forceinline__ void shift(double uc, double (&b)[NC]) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) b[i] = cs[i];
#pragma unroll
    for (int m = 0; m < NC - 1; ++m)
#pragma unroll
      for (int i = NC - 2; i >= m; --i) b[i] = fma(b[i + 1], uc, b[i]);
  }
  // Even and odd parts at K = k^2.
  __device__ __forceinline__ void parts(const double (&b)[NC], double K, double& E,
                                        double& O) const {
    constexpr int ev = (NC - 1) & ~1, od = ((NC - 2) | 1);
    E = b[ev];
#pragma unroll
    for (int e = ev - 2; e >= 0; e -= 2) E = fma(E, K, b[e]);
    O = b[od];
#pragma unroll
    for (int o = od - 2; o >= 1; o -= 2) O = fma(O, K, b[o]);
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xm, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile && NC <= 8, "Taylor-pair tiles: NC <= 8, 64 samples");
      const double um = xm * inv_h;  // tile midpoint in steps
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        double b[NC];
        shift(um + (q == 0 ? -c16 : c16), b);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) {
          double E, O;
          parts(b, pk[j] * pk[j], E, O);
          t += fma(pk[j], O, E);   // sample kSub/2 + j of the sub-tile
          t += fma(-pk[j], O, E);  // sample kSub/2 - 1 - j
          asm volatile("" : "+v"(t));  // keep program order (see Pi4)
        }
      }
      return acc + t;
    } else {
      return acc + tile<U, M>(xm, h);
    }
  }
  // Sample u of a full series tile by exactly tile_acc's operations (validation kernel).
  __device__ __forceinline__ double series_point(double xm, int u) const {
    const int q = u / kSub, w = u % kSub;
    double b[NC];
    shift(xm * inv_h + (q == 0 ? -c16 : c16), b);
    const int j = w >= kSub / 2 ? w - kSub / 2 : kSub / 2 - 1 - w;
    double E, O;
    parts(b, pk[j] * pk[j], E, O);
    return w >= kSub / 2 ? fma(pk[j], O, E) : fma(-pk[j], O, E);
  }
};

// ------------------------------------------------------------------ analytic train velocity
// v(t) = (1 - cos(t/ts)) * vs   (riemann.cpp:108-111). Integral over [0,1800] is
// dis_function(1800) = vs*(1800 - ts*sin(1800/ts)) ~= 121999.99983.
// kSeries: AngleSeries with w = 1/ts on cos; tile value vs (U - sum cos).
struct TrainVel : TileDefaults<TrainVel>, AngleSeries<8> {
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
    return (1.0 - cos(t * inv_ts)) * vs;
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double ta, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "angle series tiles are kSeriesTile samples");
      return fma(-vs, tile_sum<true>(ta * inv_ts), fma(vs, static_cast<double>(U), acc));
    } else {
      return acc + tile<U, M>(ta, h);
    }
  }
  __device__ __forceinline__ double series_point(double tm, int u) const {
    return (1.0 - point_of<true>(tm * inv_ts, u)) * vs;
  }
  // kIeee: every sample's own cos(t / ts) (trig_tile_sum, shift 1); the tile value is
  // vs (U - sum cos).
  template <int U, DivMode>
  __device__ __forceinline__ double tile(double x0, double h) const {
    const double c = trig_tile_sum<U, 1>(x0, h, ScaledAngle{inv_ts}, OcmlCos{});
    return fma(-vs, c, vs * static_cast<double>(U));
  }
  template <int U>
  __device__ __forceinline__ double ieee_point(double x0, double h, int u) const {
    return (1.0 - trig_tile_point<U, 1>(x0, h, u, ScaledAngle{inv_ts}, OcmlCos{})) * vs;
  }
};
// ocml cos for every sample (validation reference of the kIeee tile; set_trig_library).
struct TrainVelLib : TrainVel {
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
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xa, double h, double acc) const {
    static_assert(M != DivMode::kSeries, "TrainVelLib is the kIeee reference");
    return acc + tile<U, M>(xa, h);
  }
  template <int U>
  __device__ __forceinline__ double ieee_point(double x0, double h, int u) const {
    return point(fma(static_cast<double>(u), h, x0));
  }
};

// ------------------------------------------------------------------ velocity-profile table
// The 1801-sample table (14.4 KB) lives in LDS, loaded once per workgroup. Segment index is
// clamped to [0, nseg-1] so t == 1800 interpolates the last segment instead of reading
// past the end (the reference copies only 1800 of 1801 entries: cintegrate.cu:117,121).
//
// kIeee (the reference's per-sample form, cintegrate.cu:36-44): every sample forms its
// coordinate, truncates it to a segment index, clamps, re-reads v[k] and v[k+1] from LDS and
// interpolates: ~11 VALU + 2 LDS reads per sample.
// kSeries (default): a 64-sample tile almost never straddles a knot (a segment holds
// 1/h samples: 555 556 at N = 1e9 over [0, 1800], 10 000 at the reference's 1e4 samples/s),
// and inside one segment the interpolant is the straight line v(x_m + k h) = v_m + k (d h).
// The tile reads its segment once (v_m at the tile midpoint, slope D = d h), then every
// sample is that line at its own offset from a sub-tile centre: one fma per sample plus its
// accumulation (pairs at +-k share the centre and k), 2.2 VALU per sample with the tile
// set-up. A lane whose tile straddles a knot adds the kink of the next segment per sample
// (exec divergence; at N = 1e9 one wave in ~140 has such a lane, at 18e6 two in five). The
// table is read from global memory (L2-resident), not staged in LDS.
struct Table : TileDefaults<Table> {
  const double* lds;  // the table: LDS copy (kIeee) or the global array (kSeries)
  int nseg;           // number of segments = entries - 1
  static constexpr double kScale = 1.0;
  static constexpr int kPairs = 16;                 // sample pairs per sub-tile
  static constexpr int kSub = 2 * kPairs;           // 32 samples per sub-tile
  static constexpr int kSubs = 2;                   // sub-tile centres at -16, +16 steps
  static constexpr int kSeriesTile = kSub * kSubs;  // 64 samples per segment read
  double pk[kPairs];  // k_j = j + 1/2 (SGPR: VOP3 f64 ops take no literal on gfx9)
  double c16;         // sub-tile centre offset
  double hspan;       // (kSeriesTile - 1) / 2: tile midpoint to its end samples
  double inv_h;       // 1 / h (knot offsets in steps)

  __device__ __forceinline__ static double opaque_s(double v) {
    asm volatile("" : "+s"(v));
    return v;
  }
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < kPairs; ++j) pk[j] = opaque_s(j + 0.5);
    c16 = opaque_s(0.5 * kSub);
    hspan = opaque_s(0.5 * (kSeriesTile - 1));
  }
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
  __device__ __forceinline__ double point(double t) const {
    const int i = segment(t);
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
  // Segments of a tile's first and last samples.
  __device__ __forceinline__ void ends(double xm, double h, int& lo, int& hi) const {
    lo = segment(fma(-hspan, h, xm));
    hi = segment(fma(hspan, h, xm));
  }
  // Segment line of a one-segment tile: value at the midpoint and per-step slope.
  __device__ __forceinline__ void line(double xm, double h, int i, double& vm, double& D) const {
    const double v0 = lds[i];
    const double d = lds[i + 1] - v0;
    vm = fma(d, xm - static_cast<double>(i), v0);
    D = d * h;
  }
  // A tile that straddles exactly one knot (at x_k = lo + 1) is the line of segment lo with a
  // kink: v(x_m + k h) = v_m + k D + max(k - k_knot, 0) dD, dD = (d_{lo+1} - d_lo) h, k_knot =
  // (x_k - x_m) / h. Each sample costs 5 VALU instead of 2 (a per-sample segment select in
  // the reference's form costs ~15 and was most of the time at 18e6 samples, where two waves
  // in five carry such a tile). Entries lo..lo+2 are read once.
  struct Kink {
    double dD, kk;  // slope change per step, knot offset from the tile midpoint in steps
  };
  __device__ __forceinline__ Kink kink(double xm, double h, int lo, double& vm, double& D) const {
    const double v0 = lds[lo], v1 = lds[lo + 1], v2 = lds[lo + 2];
    const double d0 = v1 - v0;
    vm = fma(d0, xm - static_cast<double>(lo), v0);
    D = d0 * h;
    return {((v2 - v1) - d0) * h, (static_cast<double>(lo + 1) - xm) * inv_h};
  }
  // Sum of the tile's samples on the line (v_m, D), plus the kink when KINK.
  template <bool KINK>
  __device__ __forceinline__ double line_sum(double vm, double D, const Kink& kn) const {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kSubs; ++q) {
      const double c0 = q == 0 ? -c16 : c16;
      const double vc = fma(c0, D, vm);
      const double r = c0 - kn.kk;  // sub-tile centre relative to the knot
#pragma unroll
      for (int j = 0; j < kPairs; ++j) {
        double gp = fma(pk[j], D, vc);   // sample kSub/2 + j of the sub-tile
        double gn = fma(-pk[j], D, vc);  // sample kSub/2 - 1 - j
        if constexpr (KINK) {
          gp = fma(fmax(r + pk[j], 0.0), kn.dD, gp);
          gn = fma(fmax(r - pk[j], 0.0), kn.dD, gn);
        }
        t += gp;
        t += gn;
        asm volatile("" : "+v"(t));  // keep program order (see Pi4)
      }
    }
    return t;
  }
  template <int U, DivMode M>
  __device__ __forceinline__ double tile_acc(double xm, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(U == kSeriesTile, "segment tiles are kSubs sub-tiles of kSub samples");
      int lo, hi;
      ends(xm, h, lo, hi);
      double vm, D;
      if (lo == hi) {
        line(xm, h, lo, vm, D);
        return acc + line_sum<false>(vm, D, Kink{0.0, 0.0});
      }
      if (hi == lo + 1) {
        const Kink kn = kink(xm, h, lo, vm, D);
        return acc + line_sum<true>(vm, D, kn);
      }
      // coarse step (a tile spans several segments): per sample, rolled
      const double x0 = fma(-hspan, h, xm);
      double s0 = 0.0, s1 = 0.0;
#pragma unroll 1
      for (int u = 0; u < U; u += 2) {
        s0 += point(fma(static_cast<double>(u), h, x0));
        s1 += point(fma(static_cast<double>(u + 1), h, x0));
      }
      return acc + (s0 + s1);
    } else {
      return acc + tile<U, M>(xm, h);
    }
  }
  // Sample u of a full segment tile by exactly tile_acc's operations (validation kernel).
  __device__ __forceinline__ double series_point(double xm, double h, int u) const {
    int lo, hi;
    ends(xm, h, lo, hi);
    if (hi > lo + 1) return point(fma(static_cast<double>(u), h, fma(-hspan, h, xm)));
    double vm, D;
    Kink kn{0.0, 0.0};
    if (lo == hi) line(xm, h, lo, vm, D);
    else kn = kink(xm, h, lo, vm, D);
    const int q = u / kSub, w = u % kSub;
    const double c0 = q == 0 ? -c16 : c16;
    const double vc = fma(c0, D, vm);
    const double r = c0 - kn.kk;
    const int j = w >= kSub / 2 ? w - kSub / 2 : kSub / 2 - 1 - w;
    double g = w >= kSub / 2 ? fma(pk[j], D, vc) : fma(-pk[j], D, vc);
    if (lo != hi) g = fma(fmax(w >= kSub / 2 ? r + pk[j] : r - pk[j], 0.0), kn.dD, g);
    return g;
  }
};

}  // namespace miint
