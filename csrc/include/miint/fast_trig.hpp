// Per-sample fp64 sin / cos for the kIeee (per-point) Sin and TrainVel tiles.
//
// The reference evaluates libm/libdevice sin once per sample (riemann.cpp:37,
// cintegrate.cu:66-70). ocml's sin costs ~56 VALU per sample on gfx950 (its range reduction
// carries a Payne-Hanek path for huge arguments, and both kernel polynomials plus the
// quadrant selects run for every lane). Samples of one lane tile are consecutive, so this
// form hoists everything that only depends on the tile:
//
//  * Quadrant. n = rint(theta * 2/pi) of the tile's first and last angle; if they agree
//    (theta is monotone in the sample index, so every sample of the tile agrees) the whole
//    tile shares n, its kernel polynomial (sin for even n + shift, cos for odd) and its sign.
//    One wave covers 2048 consecutive samples, so across a wave n almost never differs and
//    the even/odd branch is skipped by exec (s_cbranch_execz) rather than evaluated masked.
//  * Cody-Waite constants (fdlibm's pio2_1 / pio2_2 / pio2_2t: pi/2 = P1 + P2 + P2T, P1 and
//    P2 with 33 significant bits): c1 = n P1 and t = n P2 are exact for |n| <= 2^20, w = n P2T.
//
// Per sample: r = theta - c1 (exact), y0 = r - t, y1 = ((r - y0) - t) - w (Fast2Sum: exact
// when |r| >= |t|), so theta - n pi/2 = y0 + y1 to ~2^-100 relative; then fdlibm's
// __kernel_sin / __kernel_cos WITH the tail y1 (< 1 ulp of the true value for |y0| <= pi/4).
// About 18 (sin) / 22 (cos) VALU per sample with the coordinate and the accumulation,
// against ~56 for ocml. A tile with |n| > kFastTrigMaxN (|theta| beyond ~1.03e5), with two
// quadrants, or with a sample whose reduced angle comes within |t| of zero (Fast2Sum's
// precondition; only the tile holding a zero of sin/cos, and only for n != 0) is evaluated
// by ocml per sample instead.
//
// Everything here is __host__ __device__ with contraction off (a pragma in every body), so
// the host build (the CPU accuracy tests against long double) runs exactly the device's
// operations.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace miint {

constexpr double kTwoOverPi = 6.36619772367581382433e-01;
constexpr double kPio2P1 = 1.57079632673412561417e+00;   // 0x3FF921FB54400000: 33 bits
constexpr double kPio2P2 = 6.07710050630396597660e-11;   // 0x3DD0B4611A600000: 33 bits
constexpr double kPio2P2T = 2.02226624879595063154e-21;  // pi/2 - P1 - P2
constexpr double kFastTrigMaxN = 65536.0;                // |theta| <~ 1.03e5

// fdlibm __kernel_sin(x, y, 1): sin(x + y) for |x| <= ~pi/4, |y| << ulp(x).
__host__ __device__ __forceinline__ double ksin(double x, double y) {
#pragma clang fp contract(off)
  const double z = x * x;
  const double v = z * x;
  const double r = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10,
                                            -2.50507602534068634195e-08),
                                     2.75573137070700676789e-06),
                              -1.98412698298579493134e-04),
                       8.33333333332248946124e-03);
  const double a = fma(-v, r, 0.5 * y);
  const double b = fma(z, a, -y);
  return x - fma(-v, -1.66666666666666324348e-01, b);
}

// fdlibm __kernel_cos(x, y): cos(x + y) for |x| <= ~pi/4, with the 1 - z/2 split that keeps
// it within 1 ulp.
__host__ __device__ __forceinline__ double kcos(double x, double y) {
#pragma clang fp contract(off)
  const double z = x * x;
  const double r = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11,
                                                       2.08757232129817482790e-09),
                                                -2.75573143513906633035e-07),
                                         2.48015872894767294178e-05),
                                  -1.38888888888741095749e-03),
                           4.16666666666666019037e-02);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + fma(z, r, -(x * y)));
}

// The per-tile part of the reduction: quadrant, kernel choice, sign and the Cody-Waite
// products. `shift` = 0 evaluates sin(theta), 1 evaluates cos(theta) = sin(theta + pi/2).
struct TrigTile {
  double c1, t, w;  // n P1 (exact), n P2 (exact), n P2T
  bool use_cos;     // kernel polynomial: cos for odd n + shift
  bool neg;         // sign of the tile's values
};

// Tile [th0, th1] (either order) -> per-tile constants; false = evaluate per sample by the
// library instead (two quadrants, |n| too large, or a reduced angle that can reach |t|).
__host__ __device__ __forceinline__ bool trig_tile(double th0, double th1, int shift,
                                                   TrigTile& q) {
#pragma clang fp contract(off)
  const double n = rint(th0 * kTwoOverPi);
  if (!(n == rint(th1 * kTwoOverPi)) || !(fabs(n) <= kFastTrigMaxN)) return false;
  q.c1 = n * kPio2P1;
  q.t = n * kPio2P2;
  q.w = n * kPio2P2T;
  const double r0 = th0 - q.c1, r1 = th1 - q.c1;
  // Fast2Sum(r, -t) needs |r| >= |t| at every sample: r is monotone, so the two ends decide
  // (same sign, both at least |t| away; n == 0 has t == 0 and always passes)
  const double at = fabs(q.t);
  if (at > 0.0 && !(fabs(r0) >= at && fabs(r1) >= at && (r0 >= 0.0) == (r1 >= 0.0)))
    return false;
  const int qq = static_cast<int>(n) + shift;
  q.use_cos = (qq & 1) != 0;
  q.neg = (qq & 2) != 0;
  return true;
}

// Kernel value (unsigned) of one sample of a trig tile.
template <bool COS>
__host__ __device__ __forceinline__ double trig_sample(double th, const TrigTile& q) {
#pragma clang fp contract(off)
  const double r = th - q.c1;
  const double y0 = r - q.t;
  const double y1 = ((r - y0) - q.t) - q.w;
  return COS ? kcos(y0, y1) : ksin(y0, y1);
}

// sin(theta + shift pi/2) of one sample, quadrant from the sample itself (host reference and
// validation: the same operations the tile runs once n is known). Returns false where the
// tile path would hand the sample to the library.
__host__ __device__ __forceinline__ bool fast_trig_point(double th, int shift, double& out) {
  TrigTile q;
  if (!trig_tile(th, th, shift, q)) return false;
  const double v = q.use_cos ? trig_sample<true>(th, q) : trig_sample<false>(th, q);
  out = q.neg ? -v : v;
  return true;
}

}  // namespace miint
