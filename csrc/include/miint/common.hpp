// miint — MI355X-native numerical-integration framework.
// Common host/device definitions: error checking, shared enums and parameter blocks.
//
// Replaces the reference's complete absence of error checking (SURVEY §2.7 B8:
// cintegrate.cu:116-133 ignores every cudaError_t, riemann.cpp/4main.c ignore MPI codes).
// Every HIP / RCCL call in this framework goes through MIINT_HIP / MIINT_RCCL, which
// throw a miint::Error carrying file:line so Python sees a real exception.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace miint {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const std::string& what, const char* file, int line) {
  throw Error(std::string(file) + ":" + std::to_string(line) + ": " + what);
}

}  // namespace miint

#define MIINT_HIP(expr)                                                                     \
  do {                                                                                      \
    hipError_t miint_e_ = (expr);                                                           \
    if (miint_e_ != hipSuccess)                                                             \
      ::miint::fail(std::string(#expr) + " -> " + hipGetErrorString(miint_e_), __FILE__,    \
                    __LINE__);                                                              \
  } while (0)

#define MIINT_CHECK(cond, msg)                                                   \
  do {                                                                           \
    if (!(cond)) ::miint::fail(std::string("check failed: ") + (msg), __FILE__, __LINE__); \
  } while (0)

namespace miint {

// ---------------------------------------------------------------------------------------
// Integrands. The reference hard-wires sin (riemann.cpp:37, cintegrate.cu:68) and the
// table interpolant (cintegrate.cu:36-44, 4main.c:262-269); BASELINE.json adds 4/(1+x^2)
// and synthetic random-coefficient polynomials. All are selectable at run time here.
// ---------------------------------------------------------------------------------------
enum class Integrand : int {
  kPi4 = 0,          // 4/(1+x^2) on [0,1] -> pi              (BASELINE.json configs 1-4)
  kSin = 1,          // sin(x) on [0,pi] -> 2                 (riemann.cpp:37, cintegrate.cu:68)
  kPoly = 2,         // sum_k c_k x^k (random-init coeffs)     (BASELINE.json "random-init coefficients")
  kTrainVel = 3,     // (1-cos(t/ts))*vs  analytic train       (riemann.cpp:103-116, dead code there)
  kTable = 4,        // linear interp of the 1801-pt profile   (cintegrate.cu:23-44, 4main.c:249-269)
};

// Point placement inside each subinterval. The reference only has the left rule
// (riemann.cpp:36 x = a + idx*h). Midpoint is offered because the left rule's truncation
// error (exactly h for 4/(1+x^2)) hides every other error source.
enum class Rule : int { kLeft = 0, kMid = 1, kRight = 2 };

// How the Pi4 kernels divide (see integrands.hpp for the derivation):
//   kSeries        per-tile v_rcp_f64 seed, per-sample exact residual e = 1 - d*s evaluated
//                  pairwise from the tile midpoint, 1/d = s(3/4 + g^2), g = 1/2 + e
//                  (2.65 VALU per sample; per point up to 4 ulp from the true value)
//   kIeee          correctly rounded division for every sample (reference path)
//   kSeriesDirect  the same series with x, d formed explicitly per sample (5 ops; A/B)
//   kSeriesExact   kSeries's residuals without the g = 1/2 + e fold: each sample's value is
//                  s (1 + e + e^2) at e's own precision, the seed residual from the exact
//                  d_m (2.68 VALU per sample; per point from the true value max 1.34 ulp /
//                  mean 0.27 ulp on profiles/r5/accuracy_ab.md's windows, max 1.42 on the
//                  bench record's 1/8-in window, <= 1.5 enforced by
//                  test_pi4_series_exact_per_point_accuracy and the record's per_point check;
//                  IEEE division per sample is 1.57 / 0.45): the headline
//                  division since round 5 (profiles/r5/accuracy_ab.md). For the other
//                  integrands (and fp32) it selects their series path.
enum class DivMode : int { kSeries = 0, kIeee = 1, kSeriesDirect = 2, kSeriesExact = 3 };

inline double rule_offset(Rule r) {
  return r == Rule::kLeft ? 0.0 : (r == Rule::kMid ? 0.5 : 1.0);
}

constexpr int kMaxPolyCoeffs = 16;

// Everything a Riemann kernel needs, passed by value (kernarg segment, lands in SGPRs).
constexpr int kSinTrig = 28;  // 8 x {cos, sin}(k_j h) + 6 x {cos, sin}(c0 h), c0 = 8, 24, ..., 88

struct RiemannParams {
  double a;             // integration lower bound
  double h;             // subinterval width (b-a)/n_total
  double off;           // rule offset in units of h (0, 0.5, 1)
  uint64_t i_begin;     // first global sample index owned by this launch (rank slice)
  uint64_t n;           // number of samples owned by this launch
  int integrand;        // Integrand
  int ncoef;            // polynomial: number of coefficients
  double coef[kMaxPolyCoeffs];  // polynomial coefficients c_0..c_{ncoef-1}
  // Polynomial series path, filled on the host by the launchers (long double): c_i h^i
  // (integrands.hpp, Poly::tile_acc)
  double coef_h[kMaxPolyCoeffs];
  double p0, p1;        // integrand parameters (train: ts, vs)
  // Sin series path, filled on the host by the launchers (long double): trig[j] = cos(k_j h),
  // trig[8 + j] = sin(k_j h) for k_j = j + 1/2 (j < 8), then cos(c0 h), sin(c0 h) for the
  // sub-tile centres c0 = 8, 24, ..., 88 (integrands.hpp, struct AngleSeries)
  double trig[kSinTrig];
  // The same table rounded to fp32 by the host (the fp32 sin / train series, integrands_f32.hpp):
  // kernel arguments, so the packed constants stay in SGPR pairs instead of VGPR copies.
  float trig32[kSinTrig];
};

}  // namespace miint
