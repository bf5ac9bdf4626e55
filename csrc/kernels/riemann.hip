// Riemann-sum kernels for gfx950 (MI355X / CDNA4).
//
// Reference behaviour being replaced:
//   cuda_function  cintegrate.cu:47-72  — 64 fat threads, 15.6 M sequential sin() each,
//                                         partials summed on the host.
//   riemann_sum    riemann.cpp:29-44    — serial host loop, int counter (overflows >2^31).
//
// Design (MI355X-first):
//   * Work unit = a tile of T consecutive samples owned by one lane (T = 32, or 64 for the
//     Pi4 series path: F::tile_len<M>()). Tiles are dealt
//     grid-stride over 64-bit indices, so N = 1e10+ is fine (fixes SURVEY B9) and every
//     launch fills all 256 CUs x 8 waves/SIMD regardless of N.
//   * Sample coordinates are formed from the integer index every tile
//     (x0 = fma(i0 + off, h, a), then fma(u, h, x0)) — no running x += h drift.
//   * Per-lane fp64 accumulation over ~60 tiles, then wave64 DPP reduction, LDS across the
//     4 waves of the workgroup, one partial per workgroup, and a fixed-order finalize
//     (two-kernel) or last-workgroup ticket (one kernel). No float atomics anywhere:
//     results are bitwise reproducible run to run.
//   * fp32 path: packed float2 math (v_pk_fma_f32), tile coordinates from an fp64 base.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <string>

#include "miint/common.hpp"
#include "miint/handoff.hpp"
#include "miint/integrands.hpp"
#include "miint/integrands_f32.hpp"
#include "miint/kernels.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {
namespace {

constexpr int B = kRiemannBlock;  // the default block; validation kernels run at it
// The integration kernels take their block size at launch (--block, SP in the reference,
// cintegrate.cu:17-18,124-127): 64, 128, 256, 512 or 1024 threads. Everything that depends
// on it reads blockDim.x; the hot tile loop itself does not.
constexpr int kMaxBlock = 1024;

// Wave-uniform 64-bit value read from one lane (two 32-bit v_readlane).
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), lane);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), lane);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Accumulate f over this launch's samples [p.i_begin, p.i_begin + p.n) into a per-lane sum.
//  * Lane g owns tiles g, g+L, g+2L, ... (L = all lanes of the grid). Consecutive lanes of a
//    wave differ by at most one round, so the loop runs a wave-uniform round count (SALU
//    counter, no per-tile VALU compare) and only one extra round is exec-masked.
//  * The tile's anchor index is carried as an exact double (integers < 2^53 are exact), so
//    a round costs one v_add_f64 + one v_fma_f64 for its coordinate.
// Accumulator type of a functor's lane sums and block reduction: fp64 everywhere except the
// all-fp32 variant (Pi4F32Acc32: fp32 lanes, v_add_f32_dpp wave sums, fp32 LDS step).
template <class F> struct AccOf { using type = double; };

// The launch's tiles over its lanes: with ntile = q * lanes + rem every lane runs q rounds and
// the first rem lanes one more. Wave-uniform, computed once per launch (one scalar 64-bit
// division) — the per-lane form (ntile - 1 - gid) / lanes + 1 was a VALU 64-bit division
// (~50 VALU + ~60 SALU) that the multi-step kernel paid again every step, together with a
// reload of blockDim.x and its wait.
// Lane indices and rem are below lanes < 2^32, so the per-wave compares are 32-bit (SALU has
// no 64-bit less-than: a 64-bit one would put the round counts, and the tile loop's exit
// test, on the VALU).
struct TileSplit {
  uint64_t lanes, q;
  uint32_t bs, rem;
};
template <int T>
__device__ __forceinline__ TileSplit tile_split(uint64_t n) {
  const uint32_t bs = blockDim.x;
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * bs;
  const uint64_t ntile = n / T;
  const uint64_t q = ntile / lanes;
  return {lanes, q, bs, static_cast<uint32_t>(ntile - q * lanes)};
}

// `block` is the workgroup's index in the sample decomposition: blockIdx.x, or the multi-step
// kernel's per-step rotated (virtual) index.
template <DivMode M, class F>
__device__ __forceinline__ typename AccOf<F>::type lane_sum(const RiemannParams& p, const F& f,
                                                            unsigned block, const TileSplit& sp) {
  using Acc = typename AccOf<F>::type;
  constexpr int T = F::template tile_len<M>();
  const uint64_t lanes = sp.lanes;
  const uint32_t b0 = block * sp.bs;
  const uint32_t g32 = b0 + threadIdx.x;
  const uint64_t gid = g32;
  const uint32_t w0 =  // the wave's first lane (SGPR)
      b0 + static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)) * kWave;
  // lane g runs q + (g < rem) rounds: every lane of the wave the first q + all_extra (a
  // count-down with a 64-bit != test: SALU), the wave's lanes below rem one more, exec-masked
  const bool all_extra = w0 + (kWave - 1) < sp.rem;  // lane 63, the wave's fewest
  const bool extra = !all_extra && g32 < sp.rem;      // a lane mask (SGPRs)
  const double base = static_cast<double>(p.i_begin) + p.off;
  const double istep = static_cast<double>(lanes * T);
  double ib = base + static_cast<double>(gid * T) + F::template anchor<T, M>();
  Acc acc = 0;
  // (readlane: left to itself, isel widens the uniform bool through a VGPR and runs the
  // counter on the VALU)
  for (uint64_t left = readlane_u64(sp.q + (all_extra ? 1 : 0), 0); left != 0; --left, ib += istep)
    acc = f.template tile_acc<T, M>(fma(ib, p.h, p.a), p.h, acc);
  if (extra) acc = f.template tile_acc<T, M>(fma(ib, p.h, p.a), p.h, acc);
  // remainder (< T samples): one per lane (a grid of fewer lanes than T loops)
  const uint64_t done = (sp.q * lanes + sp.rem) * T;
  for (uint64_t k = gid; k < p.n - done; k += lanes)
    acc += static_cast<Acc>(f.point(fma(base + static_cast<double>(done + k), p.h, p.a)));
  return acc;
}
template <DivMode M, class F>
__device__ __forceinline__ typename AccOf<F>::type lane_sum(const RiemannParams& p, const F& f,
                                                            unsigned block) {
  return lane_sum<M>(p, f, block, tile_split<F::template tile_len<M>()>(p.n));
}

constexpr int kMaxTable = 2048;  // LDS budget for a 1-D table: 16 KB

// ---------------------------------------------------------------------------- fp32 functor
// (the other integrands' fp32 functors: integrands_f32.hpp)

// 4/(1+x^2) in packed fp32 (v_pk_fma_f32 pairs). Tile base comes in as fp64 so sample
// coordinates do not collapse at 1e9 samples; in-tile offsets and all
// per-point math are fp32. Series division as in Pi4 (first order suffices: e^2 < 2^-24).
struct Pi4F32 : TileDefaults<Pi4F32> {
  static constexpr double kScale = 4.0;
  __device__ __forceinline__ double point(double xd) const {
    const float x = static_cast<float>(xd);
    return static_cast<double>(1.0f / fmaf(x, x, 1.0f));
  }
  // 1/d for 1 <= d <= 2^100, bitwise IEEE fp32 division, two samples at once: the fp32
  // sequence hipcc emits for 1.0f / d (v_div_scale x2, v_rcp_f32, one Newton step, q = 1 * r,
  // two residual corrections, v_div_fmas, v_div_fixup) without the range handling, which is
  // the identity there (as Pi4::recip_narrow); the fmas run packed. 2 v_rcp_f32 + 6
  // v_pk_fma_f32 per pair against ~11 VALU per sample. Pi4F32Wide runs the full division
  // when |x| can reach 2^49.
  __device__ __forceinline__ static f32x2 recip_narrow(f32x2 d) {
    const f32x2 one = {1.0f, 1.0f};
    const f32x2 nd = -d;
    f32x2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    r = pk_fma(pk_fma(nd, r, one), r, r);
    const f32x2 q = pk_fma(pk_fma(nd, r, one), r, r);
    return pk_fma(pk_fma(nd, q, one), r, q);
  }
  template <int UU, DivMode M>
  __device__ __forceinline__ double tile(double x0d, double h) const {
    const float x0 = static_cast<float>(x0d);
    const float hf = static_cast<float>(h);
    const f32x2 xb = {x0, x0};
    const f32x2 hh = {hf, hf};
    const f32x2 one = {1.0f, 1.0f};
    if constexpr (M == DivMode::kIeee) {
      f32x2 acc = {0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < UU; u += 2) {
        const f32x2 uu = {static_cast<float>(u), static_cast<float>(u + 1)};
        const f32x2 x = pk_fma(uu, hh, xb);
        acc += recip_narrow(pk_fma(x, x, one));
      }
      return static_cast<double>(acc.x) + static_cast<double>(acc.y);
    } else {
      const float xm = fmaf(0.5f * (UU - 1), hf, x0);
      const float dm = fmaf(xm, xm, 1.0f);
      float s = __builtin_amdgcn_rcpf(dm);
      s = fmaf(s, fmaf(-dm, s, 1.0f), s);
      const f32x2 ns = {-s, -s};
      f32x2 t = {0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < UU; u += 2) {
        const f32x2 uu = {static_cast<float>(u), static_cast<float>(u + 1)};
        const f32x2 x = pk_fma(uu, hh, xb);
        t += pk_fma(pk_fma(x, x, one), ns, one);  // e = 1 - d*s
      }
      const double sd = static_cast<double>(s);
      return sd * (static_cast<double>(UU) + (static_cast<double>(t.x) + static_cast<double>(t.y)));
    }
  }

  // Default series path, midpoint-anchored, 192-sample tiles of six 32-sample sub-tiles
  // (centres at -80, -48, ..., 48, 80 steps; e_c = e_m + c0 A + c0^2 B, A' = A + 2 c0 B: one
  // seed per 192 samples). Tile length vs overhead: 64-sample tiles spent ~29 VALU of seed,
  // coordinate and fp64 fold per 80 of pair work; at N = 1e9 on 2048 x 256 lanes, 128 / 192 /
  // 320-sample tiles ran 2.34e13 / 2.44e13 / 2.48e13 subint/s, and 320 doubled the
  // midpoint-rule error (4.1e-11 vs 2.1e-11: wider sub-tile offsets), so 192. (256 would
  // leave 7.45 tiles per lane, i.e. 8 on the busiest.) The pair residuals (e_{+k}, e_{-k}) = c_k + (k, -k) * A'
  // are one v_pk_fma_f32 (op_sel broadcasts c_k), summed by one v_pk_add_f32, and the shared
  // c_k of TWO consecutive pairs advance together by one v_pk_fma_f32 with the exact steps
  // (k_{j+2}^2 - k_j^2, k_{j+3}^2 - k_{j+1}^2) = (4j+6, 4j+10) times B: 1.25 VALU per sample.
  // In fp32 the e^2 term (< 3e-16) is far below the format's 6e-8 and is not carried.
  static constexpr int kSubLen = 32;
  static constexpr int kSubs = 6;
  template <DivMode M>
  __host__ __device__ static constexpr int tile_len() {
    return M == DivMode::kSeries ? kSubs * kSubLen : 32;
  }
  template <int UU, DivMode M>
  __device__ static constexpr double anchor() {
    return M == DivMode::kSeries ? 0.5 * (UU - 1) : 0.0;
  }
  template <int UU, DivMode M>
  __device__ __forceinline__ double tile_acc(double xmd, double h, double acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(UU == kSubs * kSubLen, "fp32 series tiles are kSubs 32-sample sub-tiles");
      const float xm = static_cast<float>(xmd);
      const float hf = static_cast<float>(h);
      const float dm = fmaf(xm, xm, 1.0f);
      float s = __builtin_amdgcn_rcpf(dm);
      s = fmaf(s, fmaf(-dm, s, 1.0f), s);
      const float em = fmaf(-dm, s, 1.0f);
      const float a = (-2.0f * hf) * xm * s;
      const float b = -(hf * hf) * s;
      const f32x2 bb = {b, b};
      const f32x2 aa = {a, a};
      const f32x2 emv = {em, em};
      // Sub-tile centre residuals and slopes, two sub-tiles per packed op:
      // (e_c, e_c') = c0 (c0 B + A) + e_m and (A', A'') = 2 c0 B + A for c0 pairs (-80, -48), ...
      f32x2 ecs[kSubs / 2], aqs[kSubs / 2];
#pragma unroll
      for (int p2 = 0; p2 < kSubs / 2; ++p2) {
        const f32x2 c0v = {(2 * p2 - 0.5f * (kSubs - 1)) * kSubLen,
                           (2 * p2 + 1 - 0.5f * (kSubs - 1)) * kSubLen};
        ecs[p2] = pk_fma(c0v, pk_fma(c0v, bb, aa), emv);
        aqs[p2] = pk_fma(c0v + c0v, bb, aa);
      }
      f32x2 t, t1;
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        const float ec = (q & 1) ? ecs[q / 2].y : ecs[q / 2].x;
        const float aq = (q & 1) ? aqs[q / 2].y : aqs[q / 2].x;
        const f32x2 av = {aq, aq};
        f32x2 cc = pk_fma(f32x2{0.25f, 2.25f}, bb, f32x2{ec, ec});  // (c_0, c_1)
#pragma unroll
        for (int j = 0; j < kSubLen / 2; j += 2) {
          const f32x2 k0 = {j + 0.5f, -(j + 0.5f)};
          const f32x2 k1 = {j + 1.5f, -(j + 1.5f)};
          const f32x2 e0 = pk_fma(k0, av, f32x2{cc.x, cc.x});  // (e_{+k_j}, e_{-k_j})
          const f32x2 e1 = pk_fma(k1, av, f32x2{cc.y, cc.y});  // (e_{+k_{j+1}}, e_{-k_{j+1}})
          // two running sums: no pk_add waits on the one before it (one sum: a dependent
          // v_pk_add_f32 chain with 20 s_nop hazard waits per tile; two: none, 39.6 -> 38.8 us
          // per 1e9, profiles/r4/fp32_ab.md)
          if (q == 0 && j == 0) {
            t = e0;
            t1 = e1;
          } else {
            t += e0;
            t1 += e1;
          }
          if (j + 2 < kSubLen / 2)
            cc = pk_fma(f32x2{4.0f * j + 6.0f, 4.0f * j + 10.0f}, bb, cc);
        }
      }
      t += t1;
      // Tile value s (U + sum e) folded in fp64: in fp32, U + sum e (|sum e| ~ U |e_m| ~ 4e-6)
      // rounds at ulp(128) = 1.5e-5 and drops the seed's own correction e_m, leaving every
      // tile at U fl(1/d_m): a -8e-9 relative bias at N = 1e9 (reproduced on the host by a
      // numpy emulation of this tile). Folded in fp64 the fp32 path lands on the fp64 sum.
      return fma(static_cast<double>(s), static_cast<double>(UU) + static_cast<double>(t.x + t.y),
                 acc);
    } else {
      return acc + tile<UU, M>(xmd, h);
    }
  }
};
// fp32 4/(1+x^2) by the library's full IEEE division, for kIeee launches whose coordinates can
// reach |x| >= 2^49 (the dispatcher picks it, as Pi4Wide for fp64).
struct Pi4F32Wide : Pi4F32 {
  template <int UU, DivMode M>
  __device__ __forceinline__ double tile(double x0d, double h) const {
    static_assert(M == DivMode::kIeee, "wide-domain fp32 Pi4 runs IEEE division only");
    const float x0 = static_cast<float>(x0d);
    const float hf = static_cast<float>(h);
    float acc0 = 0.0f, acc1 = 0.0f;
#pragma unroll
    for (int u = 0; u < UU; u += 2) {  // the same pairing as Pi4F32::tile
      const float xa = fmaf(static_cast<float>(u), hf, x0);
      const float xb = fmaf(static_cast<float>(u + 1), hf, x0);
      acc0 += 1.0f / fmaf(xa, xa, 1.0f);
      acc1 += 1.0f / fmaf(xb, xb, 1.0f);
    }
    return static_cast<double>(acc0) + static_cast<double>(acc1);
  }
  template <int UU, DivMode M>
  __device__ __forceinline__ double tile_acc(double x0d, double h, double acc) const {
    return acc + tile<UU, M>(x0d, h);
  }
};
constexpr double kPi4F32NarrowMaxX = 0x1p49;

// The same samples as Pi4F32, accumulated in fp32 all the way to the workgroup partial
// (DType::kF32Acc32): the tile value s (U + sum e) is formed and added in fp32, lanes reduce
// with v_add_f32_dpp and the block step runs in fp32. What this drops is the fp64 fold
// Pi4F32 keeps (see Pi4F32::tile_acc): measured against it in profiles/r3/fp32_accum.jsonl.
struct Pi4F32Acc32 : Pi4F32 {
  template <int UU, DivMode M>
  __device__ __forceinline__ float tile_acc(double xmd, double h, float acc) const {
    if constexpr (M == DivMode::kSeries) {
      static_assert(UU == kSubs * kSubLen, "fp32 series tiles are kSubs 32-sample sub-tiles");
      const float xm = static_cast<float>(xmd);
      const float hf = static_cast<float>(h);
      const float dm = fmaf(xm, xm, 1.0f);
      float s = __builtin_amdgcn_rcpf(dm);
      s = fmaf(s, fmaf(-dm, s, 1.0f), s);
      const float em = fmaf(-dm, s, 1.0f);
      const float a = (-2.0f * hf) * xm * s;
      const float b = -(hf * hf) * s;
      const f32x2 bb = {b, b};
      const f32x2 aa = {a, a};
      const f32x2 emv = {em, em};
      f32x2 ecs[kSubs / 2], aqs[kSubs / 2];
#pragma unroll
      for (int p2 = 0; p2 < kSubs / 2; ++p2) {
        const f32x2 c0v = {(2 * p2 - 0.5f * (kSubs - 1)) * kSubLen,
                           (2 * p2 + 1 - 0.5f * (kSubs - 1)) * kSubLen};
        ecs[p2] = pk_fma(c0v, pk_fma(c0v, bb, aa), emv);
        aqs[p2] = pk_fma(c0v + c0v, bb, aa);
      }
      f32x2 t, t1;
#pragma unroll
      for (int q = 0; q < kSubs; ++q) {
        const float ec = (q & 1) ? ecs[q / 2].y : ecs[q / 2].x;
        const float aq = (q & 1) ? aqs[q / 2].y : aqs[q / 2].x;
        const f32x2 av = {aq, aq};
        f32x2 cc = pk_fma(f32x2{0.25f, 2.25f}, bb, f32x2{ec, ec});
#pragma unroll
        for (int j = 0; j < kSubLen / 2; j += 2) {
          const f32x2 k0 = {j + 0.5f, -(j + 0.5f)};
          const f32x2 k1 = {j + 1.5f, -(j + 1.5f)};
          const f32x2 e0 = pk_fma(k0, av, f32x2{cc.x, cc.x});
          const f32x2 e1 = pk_fma(k1, av, f32x2{cc.y, cc.y});
          if (q == 0 && j == 0) {  // two running sums, as Pi4F32::tile_acc
            t = e0;
            t1 = e1;
          } else {
            t += e0;
            t1 += e1;
          }
          if (j + 2 < kSubLen / 2)
            cc = pk_fma(f32x2{4.0f * j + 6.0f, 4.0f * j + 10.0f}, bb, cc);
        }
      }
      t += t1;
      return fmaf(s, static_cast<float>(UU) + (t.x + t.y), acc);  // all fp32
    } else {
      const float x0 = static_cast<float>(xmd);
      const float hf = static_cast<float>(h);
      const f32x2 xb = {x0, x0}, hh = {hf, hf}, one = {1.0f, 1.0f};
      f32x2 a2 = {0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < UU; u += 2) {
        const f32x2 uu = {static_cast<float>(u), static_cast<float>(u + 1)};
        const f32x2 x = pk_fma(uu, hh, xb);
        a2 += recip_narrow(pk_fma(x, x, one));
      }
      return acc + (a2.x + a2.y);
    }
  }
};
template <> struct AccOf<Pi4F32Acc32> { using type = float; };

// The host's series validity checks (series_ok: kSeriesHalfSpan * h <= 2e-6; series_ok_f32
// with kSeriesHalfSpanF32) must bound the farthest sample offset of each Pi4 series tile.
static_assert(2 * AngleSeries<12>::kPairs + 12 == kSinTrig, "trig table sized for Sin");
static_assert(Pi4::kSeriesTile / 2 == kSeriesHalfSpan &&
                  Pi4F32::kSubs * Pi4F32::kSubLen / 2 == kSeriesHalfSpanF32,
              "kSeriesHalfSpan(F32) must be half the Pi4 series tile lengths");

// ---------------------------------------------------------------------------- functor makers
// Each integrand gets its own kernel instantiation (own register allocation); only the
// table integrand reserves LDS.
template <class F> struct Maker;
template <> struct Maker<Pi4> {
  static constexpr int kLds = 1;
  __device__ static Pi4 make(const RiemannParams&, const double*, int, double*) {
    Pi4 f;
    f.init();
    return f;
  }
};
template <> struct Maker<Pi4Wide> {
  static constexpr int kLds = 1;
  __device__ static Pi4Wide make(const RiemannParams&, const double*, int, double*) { return {}; }
};
template <> struct Maker<Pi4F32Wide> {
  static constexpr int kLds = 1;
  __device__ static Pi4F32Wide make(const RiemannParams&, const double*, int, double*) {
    return {};
  }
};
template <> struct Maker<Pi4F32Acc32> {
  static constexpr int kLds = 1;
  __device__ static Pi4F32Acc32 make(const RiemannParams&, const double*, int, double*) {
    return {};
  }
};
template <> struct Maker<Pi4F32> {
  static constexpr int kLds = 1;
  __device__ static Pi4F32 make(const RiemannParams&, const double*, int, double*) { return {}; }
};
template <> struct Maker<Sin> {
  static constexpr int kLds = 1;
  __device__ static Sin make(const RiemannParams& p, const double*, int, double*) {
    Sin f;
    f.init(p.trig);
    return f;
  }
};
template <> struct Maker<SinLib> {
  static constexpr int kLds = 1;
  __device__ static SinLib make(const RiemannParams&, const double*, int, double*) { return {}; }
};
template <int NC> struct Maker<Poly<NC>> {
  static constexpr int kLds = 1;
  __device__ static Poly<NC> make(const RiemannParams& p, const double*, int, double*) {
    Poly<NC> f;
    f.init(p.coef, p.ncoef);
    return f;
  }
};
template <> struct Maker<TrainVel> {
  static constexpr int kLds = 1;
  __device__ static TrainVel make(const RiemannParams& p, const double*, int, double*) {
    TrainVel f;
    f.init_trig(p.trig);
    f.inv_ts = 1.0 / p.p0;
    f.vs = p.p1;
    return f;
  }
};
template <> struct Maker<TrainVelLib> {
  static constexpr int kLds = 1;
  __device__ static TrainVelLib make(const RiemannParams& p, const double*, int, double*) {
    TrainVelLib f;
    f.inv_ts = 1.0 / p.p0;
    f.vs = p.p1;
    return f;
  }
};
template <> struct Maker<SinF32> {
  static constexpr int kLds = 1;
  __device__ static SinF32 make(const RiemannParams& p, const double*, int, double*) {
    SinF32 f;
    f.init(p.trig32);
    return f;
  }
};
template <> struct Maker<TrainVelF32> {
  static constexpr int kLds = 1;
  __device__ static TrainVelF32 make(const RiemannParams& p, const double*, int, double*) {
    TrainVelF32 f;
    f.init_trig(p.trig32);
    f.inv_ts = 1.0 / p.p0;
    f.vs = p.p1;
    return f;
  }
};
template <int NC> struct Maker<PolyF32<NC>> {
  static constexpr int kLds = 1;
  __device__ static PolyF32<NC> make(const RiemannParams& p, const double*, int, double*) {
    PolyF32<NC> f;
    f.init(p.coef, p.ncoef);
    return f;
  }
};
template <> struct Maker<TableF32> {
  static constexpr int kLds = kMaxTable;
  __device__ static TableF32 make(const RiemannParams&, const double* table, int n, double* lds) {
    for (int i = threadIdx.x; i < n; i += static_cast<int>(blockDim.x)) lds[i] = table[i];
    __syncthreads();
    TableF32 f;
    f.tab = lds;
    f.nseg = n - 1;
    return f;
  }
};
template <> struct Maker<Table> {
  static constexpr int kLds = kMaxTable;
  __device__ static Table make(const RiemannParams&, const double* table, int n, double* lds) {
    for (int i = threadIdx.x; i < n; i += static_cast<int>(blockDim.x)) lds[i] = table[i];
    __syncthreads();
    Table f{{}, lds, n - 1};
    f.init();
    return f;
  }
};

// Functor construction and LDS size per (division mode, integrand). The table's segment-line
// tiles read two or three entries per 64 samples, so they read the (L2-resident, 14.4 KB)
// table from global memory instead of staging all of it in every workgroup's LDS.
template <DivMode M, class F>
constexpr int lds_words() {
  if constexpr ((__is_same(F, Table) || __is_same(F, TableF32)) && M == DivMode::kSeries) return 1;
  else return Maker<F>::kLds;
}
template <class F> struct IsPoly { static constexpr bool value = false; };
template <int NC> struct IsPoly<Poly<NC>> { static constexpr bool value = true; };
template <int NC> struct IsPoly<PolyF32<NC>> { static constexpr bool value = true; };
template <class F> struct IsPolyF64 { static constexpr bool value = false; };
template <int NC> struct IsPolyF64<Poly<NC>> { static constexpr bool value = true; };

template <DivMode M, class F>
__device__ __forceinline__ F make_functor(const RiemannParams& p, const double* table, int n,
                                          double* lds) {
  if constexpr (IsPoly<F>::value && M == DivMode::kSeries) {
    F f = Maker<F>::make(p, table, n, lds);
    f.init_series(p.coef_h, p.ncoef, p.h);
    return f;
  } else if constexpr (__is_same(F, Pi4) && M != DivMode::kSeries && M != DivMode::kSeriesExact) {
    return Pi4{};  // the register-pinned pair tables (Pi4::init) serve only the series tiles
  } else if constexpr (__is_same(F, Table) && M == DivMode::kSeries) {
    Table f{{}, table, n - 1};
    f.init();
    f.inv_h = 1.0 / p.h;
    return f;
  } else if constexpr (__is_same(F, TableF32) && M == DivMode::kSeries) {
    TableF32 f;
    f.tab = table;
    f.nseg = n - 1;
    f.inv_h = 1.0 / p.h;
    return f;
  } else {
    return Maker<F>::make(p, table, n, lds);
  }
}

// The default grid (default_riemann_shape) deals 8 workgroups of 4 waves to every CU, i.e.
// 8 waves per SIMD in ONE resident round. A kernel that fits fewer (more than 64 VGPRs or
// ~96 SGPRs per wave) leaves 1/8 or more of the workgroups for a second, nearly empty round,
// and the scheduler does not trade registers for occupancy by itself: the table's segment
// tiles took 98 VGPRs (4 waves/SIMD), the train series 90 SGPRs + 66 VGPRs (7 waves/SIMD).
// Those instantiations get amdgpu_waves_per_eu(8). The ones that already fit 8 keep the
// unhinted kernel: the hint also changes their allocation (Pi4 series: 8 more VALU per tile,
// its k^2 constants moved from SGPRs to VGPR copies; sin series: 12 bytes of scratch).
#define kFullOccupancy __attribute__((amdgpu_waves_per_eu(8, 8)))
template <DivMode M, class F>
constexpr bool occupancy_hint() {
  if constexpr (__is_same(F, Pi4)) return M == DivMode::kSeriesDirect;
  else if constexpr (__is_same(F, Pi4F32) || __is_same(F, Pi4F32Wide) ||
                     __is_same(F, Pi4F32Acc32))
    return M == DivMode::kIeee;
  else if constexpr (__is_same(F, SinLib) || __is_same(F, TrainVelLib)) return true;
  else if constexpr (__is_same(F, Sin)) return M == DivMode::kIeee;
  else if constexpr (__is_same(F, PolyF32<16>)) return true;
  else if constexpr (IsPoly<F>::value) return M == DivMode::kSeries;
  else if constexpr (__is_same(F, SinF32) || __is_same(F, TrainVelF32))
    return M == DivMode::kSeries;
  else return __is_same(F, TrainVel) || __is_same(F, Table) || __is_same(F, TableF32);
}

// Partials kernel: one fp64 partial per workgroup.
template <DivMode M, class F>
__device__ __forceinline__ void partials_body(const RiemannParams& p, const double* table,
                                              int table_n, double* partials) {
  using Acc = typename AccOf<F>::type;
  __shared__ Acc red[kMaxBlock / kWave];
  __shared__ double lds[lds_words<M, F>()];
  const F f = make_functor<M, F>(p, table, table_n, lds);
  const double s = static_cast<double>(block_sum_dyn(lane_sum<M>(p, f, blockIdx.x), red));
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) void riemann_kernel(RiemannParams p, const double* table,
                                                    int table_n, double* partials) {
  partials_body<M, F>(p, table, table_n, partials);
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) kFullOccupancy void riemann_kernel_o8(RiemannParams p,
                                                                      const double* table,
                                                                      int table_n,
                                                                      double* partials) {
  partials_body<M, F>(p, table, table_n, partials);
}

// ---------------------------------------------------------------------------- finalize
// Same width and order as the fused kernel's last-workgroup sum (launched at the plan's
// block size bs: partial i folded into thread i % bs in increasing i), so both paths are
// bitwise identical.
__device__ __forceinline__ double ordered_sum(const double* partials, int n, double* red) {
  return block_sum_dyn(ordered_partials<0, false>(partials, n), red);
}

__global__ __launch_bounds__(kMaxBlock) void finalize_kernel(const double* partials, int n,
                                                             double scale, double* out) {
  __shared__ double red[kMaxBlock / kWave];
  const double s = ordered_sum(partials, n, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// ---------------------------------------------------------------------------- fused (ticket)
// One launch: partials, then the last-workgroup hand-off of handoff.hpp (write-once slots,
// two-level ticket, index-ordered sum, re-arm) — bitwise identical to partials + finalize.
template <DivMode M, class F>
__device__ __forceinline__ void fused_body(const RiemannParams& p, const double* table,
                                           int table_n, double* partials, unsigned int* ticket,
                                           double scale, double* out) {
  using Acc = typename AccOf<F>::type;
  __shared__ double red[kMaxBlock / kWave];
  __shared__ Acc red_acc[__is_same(Acc, double) ? 1 : kMaxBlock / kWave];
  __shared__ double lds[lds_words<M, F>()];
  __shared__ int is_last;
  const F f = make_functor<M, F>(p, table, table_n, lds);
  double s;
  if constexpr (__is_same(Acc, double)) s = block_sum_dyn(lane_sum<M>(p, f, blockIdx.x), red);
  else s = static_cast<double>(block_sum_dyn(lane_sum<M>(p, f, blockIdx.x), red_acc));
  if (!publish_and_ticket(s, partials, ticket, blockIdx.x, gridDim.x, &is_last)) return;
  const double v = ordered_partials<0, true>(partials, static_cast<int>(gridDim.x));
  rearm_slots<0>(partials, static_cast<int>(gridDim.x));
  const double tot = block_sum_dyn(v, red);
  if (threadIdx.x == 0) out[0] = tot * scale;
  rearm_ticket(ticket, gridDim.x);
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) void riemann_fused_kernel(RiemannParams p, const double* table,
                                                          int table_n, double* partials,
                                                          unsigned int* ticket, double scale,
                                                          double* out) {
  fused_body<M, F>(p, table, table_n, partials, ticket, scale, out);
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) kFullOccupancy void riemann_fused_kernel_o8(
    RiemannParams p, const double* table, int table_n, double* partials, unsigned int* ticket,
    double scale, double* out) {
  fused_body<M, F>(p, table, table_n, partials, ticket, scale, out);
}

// ---------------------------------------------------------------------------- chained finalize
// Graph batches of steps: kernel k writes step k's partials (plain stores, no ticket) and its
// LAST workgroup first sums step k-1's partials (written by kernel k-1; the kernel boundary
// makes them visible) into step k-1's result, in finalize_kernel's order (bitwise equal to
// the fused and two-kernel paths). Lanes with the highest ids own one tile round fewer
// whenever the tiles do not divide evenly over the grid (N = 1e9: 14 rounds instead of 15,
// ~5 us of slack), so that workgroup absorbs the ~2 us of dependent loads inside the
// kernel instead of every launch ending with the ticket round trips (fused 76.2 us vs
// partials-only 73.6 us at N = 1e9). A trailing finalize_kernel closes the batch.
template <DivMode M, class F>
__device__ __forceinline__ void chained_body(const RiemannParams& p, const double* table,
                                             int table_n, double* partials, const double* prev,
                                             int nprev, double scale, double* out_prev) {
  __shared__ double red[kMaxBlock / kWave];
  __shared__ double lds[lds_words<M, F>()];
  if (prev != nullptr && blockIdx.x == gridDim.x - 1) {
    const double tot = block_sum_dyn(ordered_partials<0, false>(prev, nprev), red);
    if (threadIdx.x == 0) out_prev[0] = tot * scale;
    __syncthreads();  // red is reused below
  }
  const F f = make_functor<M, F>(p, table, table_n, lds);
  double s;
  if constexpr (__is_same(typename AccOf<F>::type, double)) {
    s = block_sum_dyn(lane_sum<M>(p, f, blockIdx.x), red);
  } else {
    __shared__ typename AccOf<F>::type red_acc[kMaxBlock / kWave];
    s = static_cast<double>(block_sum_dyn(lane_sum<M>(p, f, blockIdx.x), red_acc));
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) void riemann_chained_kernel(RiemannParams p, const double* table,
                                                            int table_n, double* partials,
                                                            const double* prev, int nprev,
                                                            double scale, double* out_prev) {
  chained_body<M, F>(p, table, table_n, partials, prev, nprev, scale, out_prev);
}
template <DivMode M, class F>
__global__ __launch_bounds__(kMaxBlock) kFullOccupancy void riemann_chained_kernel_o8(
    RiemannParams p, const double* table, int table_n, double* partials, const double* prev,
    int nprev, double scale, double* out_prev) {
  chained_body<M, F>(p, table, table_n, partials, prev, nprev, scale, out_prev);
}

// ---------------------------------------------------------------------------- multi-step
// K complete integrations in ONE launch (graph batches with RiemannConfig::multistep). A
// chained batch pays every step's launch ramp, tail drain and end-of-kernel release; here the
// workgroups stay resident for the whole batch. At step s every workgroup computes the
// partial of its VIRTUAL block (blockIdx + s * rot) mod grid and stores it into
// partials[s][virtual block] — no ticket, no wait, no hand-off inside the launch. The
// rotation moves the blocks that own one tile round more than the rest (the first `rot`,
// lane_sum) to other workgroups every step, so over a batch every workgroup does the same
// work. multistep_close_kernel then closes all K steps at once (one workgroup per step,
// index-ordered sums, the kernel boundary orders the partials): every step's value is the
// fused / chained / two-kernel value at the same grid, bit for bit (a partial depends only on
// its virtual block). The grid should be resident as a whole (riemann_multistep_grid): a
// second round of workgroups would start only after the first finished every step.
// Each step re-derives its sample coordinates from p.a laundered through an empty asm, so
// nothing of a step is loop-invariant: no step's work can be hoisted out of the loop or shared
// with another, K steps are K full integrations.
// Steps per block sum (A/B knob, MIINT_MS_CHUNK; fp64 Pi4 kernels only): C steps' lane sums
// are kept in registers and summed over the block together (block_sums_dyn: C interleaved
// DPP chains, one barrier per C steps), each step's value bitwise the one-at-a-time sum's.
// At the 1/8 share (one wave per SIMD) C = 4 cut a wave's waits from 4.6 % to 3.5 % of its
// cycles, but interleaved A/Bs put its time within the spread of C = 1 at every share and at
// G = 1 (profiles/r6/roofline_share.md, batch_tail.md), and it takes the headline kernel
// from 62 to 69 VGPRs: the default stays 1 (the other integrands always; the polynomial's
// kernel would lose a wave per SIMD at 79 VGPRs).
#ifndef MIINT_MS_CHUNK
#define MIINT_MS_CHUNK 1
#endif
template <class F>
constexpr int ms_chunk() {
  return __is_same(F, Pi4) ? MIINT_MS_CHUNK : 1;
}

template <DivMode M, class F, bool CLOSE>
__device__ __forceinline__ void multistep_body(const RiemannParams& p, const double* table,
                                               int table_n, double* partials, int steps,
                                               unsigned rot, unsigned* ticket, double scale,
                                               double* out) {
  using Acc = typename AccOf<F>::type;
  constexpr int C = ms_chunk<F>();
  // The block sum's LDS slots alternate between block sums: sum k + 2 writes red[k & 1] only
  // after every wave passed sum k + 1's barrier, which wave 0 reaches after its sum-k reads
  // — so no second barrier per sum, and waves 1-3 start the next step while wave 0 finishes
  // the cross-wave sum.
  __shared__ double red[2][C * (kMaxBlock / kWave)];
  __shared__ Acc red_acc[2][__is_same(Acc, double) ? 1 : C * (kMaxBlock / kWave)];
  __shared__ double lds[lds_words<M, F>()];
  const F f = make_functor<M, F>(p, table, table_n, lds);
  const unsigned nb = gridDim.x;
  const TileSplit sp = tile_split<F::template tile_len<M>()>(p.n);  // the same every step
  unsigned vb = blockIdx.x;
  unsigned seq = 0;  // block sums so far (LDS buffer seq & 1)
  int s = 0;
  if constexpr (C > 1) {
    for (; s + C <= steps; s += C, ++seq) {
      const unsigned vb0 = vb;
      Acc l[C];
#pragma unroll
      for (int k = 0; k < C; ++k) l[k] = Acc(0);
#pragma unroll 1
      for (int c = 0; c < C; ++c) {
        RiemannParams q = p;
        asm volatile("" : "+s"(q.a));  // a fresh value every step (no instructions)
        const Acc x = lane_sum<M>(q, f, vb, sp);
#pragma unroll
        for (int k = 0; k < C; ++k) l[k] = k == c ? x : l[k];  // uniform select, no scratch
        vb += rot;
        if (vb >= nb) vb -= nb;
      }
      Acc v[C];
      if constexpr (__is_same(Acc, double)) block_sums_dyn<C>(l, red[seq & 1], v);
      else block_sums_dyn<C>(l, red_acc[seq & 1], v);
      if (threadIdx.x == 0) {
        unsigned w = vb0;
#pragma unroll
        for (int k = 0; k < C; ++k) {
          const double vk = static_cast<double>(v[k]);
          if constexpr (CLOSE) slot_store(&partials[static_cast<size_t>(s + k) * nb + w], vk);
          else partials[static_cast<size_t>(s + k) * nb + w] = vk;
          w += rot;
          if (w >= nb) w -= nb;
        }
      }
    }
  }
  for (; s < steps; ++s, ++seq) {
    RiemannParams q = p;
    asm volatile("" : "+s"(q.a));  // a fresh value every step (no instructions)
    double v;
    if constexpr (__is_same(Acc, double)) v = block_sum_dyn(lane_sum<M>(q, f, vb, sp), red[seq & 1]);
    else v = static_cast<double>(block_sum_dyn(lane_sum<M>(q, f, vb, sp), red_acc[seq & 1]));
    if (threadIdx.x == 0) {
      // in-launch close: write-through, read by other workgroups' closers in this launch
      if constexpr (CLOSE) slot_store(&partials[static_cast<size_t>(s) * nb + vb], v);
      else partials[static_cast<size_t>(s) * nb + vb] = v;
    }
    vb += rot;
    if (vb >= nb) vb -= nb;
  }
  if constexpr (CLOSE) {
    __shared__ int role;
    __syncthreads();  // red[] is the close's block-sum scratch: every wave past its last read
    close_batch_in_launch(partials, nb, steps, ticket, scale, out, red[0], &role);
  }
}
template <DivMode M, class F, bool CLOSE>
__global__ __launch_bounds__(kMaxBlock) void riemann_multistep_kernel(
    RiemannParams p, const double* table, int table_n, double* partials, int steps,
    unsigned rot, unsigned* ticket, double scale, double* out) {
  multistep_body<M, F, CLOSE>(p, table, table_n, partials, steps, rot, ticket, scale, out);
}
template <DivMode M, class F, bool CLOSE>
__global__ __launch_bounds__(kMaxBlock) kFullOccupancy void riemann_multistep_kernel_o8(
    RiemannParams p, const double* table, int table_n, double* partials, int steps,
    unsigned rot, unsigned* ticket, double scale, double* out) {
  multistep_body<M, F, CLOSE>(p, table, table_n, partials, steps, rot, ticket, scale, out);
}
// The step loop's state lifts every multi-step kernel to 106 SGPRs: 7 waves per SIMD. Those
// with few VGPRs take the 8-wave hint instead (the extra SGPRs go to VGPR lanes, outside the
// tile loop).
// The table's segment tiles take the 8-wave hint too: without it they held 106 VGPRs in the
// multi-step kernel (4 waves per SIMD, slower than chained launches: profiles/r3/
// multistep_ab.md); with it 42 (segment tiles) / 58 (per sample) VGPRs, 78 SGPRs, no
// scratch, and the batch runs 5.6 % faster than chained (profiles/r6/batch_tail.md).
template <DivMode M, class F>
constexpr bool multistep_o8() {
  if constexpr (__is_same(F, Table) || __is_same(F, TableF32)) return true;
  return M == DivMode::kIeee && (__is_same(F, Pi4F32) || __is_same(F, Pi4F32Wide) ||
                                 __is_same(F, Pi4F32Acc32));
}
// Instantiations whose in-launch close would not fit their register budget (under the
// 8-wave hint the close code spills 28 bytes: the table's tiles, the fp32 IEEE tiles): their
// plans close batches with the closing kernel whatever RiemannConfig::close says.
template <DivMode M, class F>
constexpr bool multistep_close_ok() {
  return !multistep_o8<M, F>();
}
// Instantiations the multi-step batch does not pay for (profiles/r3/multistep_ab.md): the
// fp64 per-sample IEEE division tiles ran 3.3 % slower even at 8 waves (371 vs 359 us).
template <DivMode M, class F>
constexpr bool multistep_pays() {
  return !(M == DivMode::kIeee && (__is_same(F, Pi4) || __is_same(F, Pi4Wide)));
}

// Closes a multi-step launch: workgroup s sums step s's partials in index order (finalize
// order) into out[s].
__global__ __launch_bounds__(kMaxBlock) void multistep_close_kernel(const double* partials,
                                                                   int nb, double scale,
                                                                   double* out) {
  __shared__ double red[kMaxBlock / kWave];
  const double t = ordered_partials<0, false>(partials + static_cast<size_t>(blockIdx.x) * nb, nb);
  const double tot = block_sum_dyn(t, red);
  if (threadIdx.x == 0) out[blockIdx.x] = tot * scale;
}

// ---------------------------------------------------------------------------- validation
// Writes every sample's f value exactly as the hot tile path evaluates it (one lane per
// tile), so tests can compare the series division point by point against IEEE division.
template <DivMode M, class F>
__global__ __launch_bounds__(B) void point_values_kernel(RiemannParams p, const double* table,
                                                         int table_n, double* out) {
  constexpr int T = F::template tile_len<M>();
  __shared__ double lds[lds_words<M, F>()];
  const F f = make_functor<M, F>(p, table, table_n, lds);
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * B + threadIdx.x;
  if (t * T >= p.n) return;
  const double x0 = fma(static_cast<double>(p.i_begin) + p.off + static_cast<double>(t * T),
                        p.h, p.a);
  const double xm = fma(0.5 * (T - 1), p.h, x0);
  const bool full = (t + 1) * T <= p.n;  // a partial tile is summed point by point
  for (int u = 0; u < T && t * T + u < p.n; ++u) {
    const double x = fma(static_cast<double>(u), p.h, x0);
    double v;
    if constexpr (M == DivMode::kSeries && __is_same(F, Pi4)) {
      // exactly the operations Pi4::tile_acc applies to sample u
      v = full ? f.series_point(xm, p.h, u) : f.point(x);
    } else if constexpr (M == DivMode::kSeriesExact && __is_same(F, Pi4)) {
      v = full ? f.series_exact_point(xm, p.h, u) : f.point(x);
    } else if constexpr (M == DivMode::kSeries && IsPolyF64<F>::value) {
      v = full ? f.series_point(xm, u) : f.point(x);
    } else if constexpr (M == DivMode::kSeries && __is_same(F, Table)) {
      v = full ? f.series_point(xm, p.h, u) : f.point(x);
    } else if constexpr (M == DivMode::kSeries && (__is_same(F, Sin) || __is_same(F, TrainVel))) {
      v = full ? f.series_point(xm, u) : f.point(x);
    } else if constexpr (M == DivMode::kSeriesDirect && __is_same(F, Pi4)) {
      const Pi4::Seed sd = Pi4::seed(xm, p.h);
      const double e = fma(-fma(x, x, 1.0), sd.s, 1.0);
      v = fma(sd.s, e + e * e, sd.s);
    } else if constexpr (M == DivMode::kIeee && __is_same(F, Pi4)) {
      v = full ? Pi4::recip_narrow(fma(x, x, 1.0)) : f.point(x);  // as Pi4::tile<U, kIeee>
    } else if constexpr (M == DivMode::kIeee &&
                         (__is_same(F, Sin) || __is_same(F, SinLib) ||
                          __is_same(F, TrainVel) || __is_same(F, TrainVelLib))) {
      v = full ? f.template ieee_point<T>(x0, p.h, u) : f.point(x);  // as F::tile<T, kIeee>
    } else {
      v = f.point(x);
    }
    out[t * T + u] = v * F::kScale;
  }
}

// Validation: Pi4::recip_narrow of arbitrary operands (tests compare it bit for bit with
// IEEE division).
__global__ __launch_bounds__(B) void recip_narrow_kernel(const double* d, uint64_t n,
                                                         double* out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * B;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * B + threadIdx.x; i < n; i += stride)
    out[i] = Pi4::recip_narrow(d[i]);
}
__global__ __launch_bounds__(B) void recip_narrow_f32_kernel(const float* d, uint64_t n,
                                                             float* out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * B;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * B + threadIdx.x; i < n; i += stride)
    out[i] = Pi4F32::recip_narrow(f32x2{d[i], d[i]}).x;
}

template <DivMode M, class F>
void launch_partials_t(const RiemannParams& p, LaunchShape shape, const double* table,
                       int table_n, double* partials, hipStream_t stream) {
  if constexpr (occupancy_hint<M, F>())
    riemann_kernel_o8<M, F><<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials);
  else
    riemann_kernel<M, F><<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials);
}
template <DivMode M, class F>
void launch_fused_t(const RiemannParams& p, LaunchShape shape, const double* table, int table_n,
                    double* partials, unsigned* ticket, double scale, double* out,
                    hipStream_t stream) {
  if constexpr (occupancy_hint<M, F>())
    riemann_fused_kernel_o8<M, F>
        <<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials, ticket, scale, out);
  else
    riemann_fused_kernel<M, F>
        <<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials, ticket, scale, out);
}

template <DivMode M, class F>
void launch_chained_t(const RiemannParams& p, LaunchShape shape, const double* table,
                      int table_n, double* partials, const double* prev, int nprev, double scale,
                      double* out_prev, hipStream_t stream) {
  if constexpr (occupancy_hint<M, F>())
    riemann_chained_kernel_o8<M, F><<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials,
                                                                  prev, nprev, scale, out_prev);
  else
    riemann_chained_kernel<M, F><<<shape.grid, shape.block, 0, stream>>>(p, table, table_n, partials,
                                                               prev, nprev, scale, out_prev);
}

template <DivMode M, class F, bool CLOSE>
void launch_multistep_c(const RiemannParams& p, LaunchShape shape, const double* table,
                        int table_n, double* partials, int steps, unsigned rot,
                        unsigned* ticket, double scale, double* out, hipStream_t stream) {
  if constexpr (multistep_o8<M, F>())
    riemann_multistep_kernel_o8<M, F, CLOSE><<<shape.grid, shape.block, 0, stream>>>(
        p, table, table_n, partials, steps, rot, ticket, scale, out);
  else
    riemann_multistep_kernel<M, F, CLOSE><<<shape.grid, shape.block, 0, stream>>>(
        p, table, table_n, partials, steps, rot, ticket, scale, out);
}
// ticket != nullptr: the in-launch close (close_batch_in_launch) stores the step values;
// otherwise the caller closes the batch with multistep_close_kernel.
template <DivMode M, class F>
void launch_multistep_t(const RiemannParams& p, LaunchShape shape, const double* table,
                        int table_n, double* partials, int steps, unsigned rot,
                        unsigned* ticket, double scale, double* out, hipStream_t stream) {
  if constexpr (multistep_pays<M, F>()) {
    if constexpr (multistep_close_ok<M, F>()) {
      if (ticket) {
        launch_multistep_c<M, F, true>(p, shape, table, table_n, partials, steps, rot, ticket,
                                       scale, out, stream);
        return;
      }
    } else {
      MIINT_CHECK(ticket == nullptr, "this integrand closes multi-step batches by a kernel");
    }
    launch_multistep_c<M, F, false>(p, shape, table, table_n, partials, steps, rot, ticket,
                                    scale, out, stream);
  } else {
    fail("this integrand/division keeps chained batches (no multi-step kernel)", __FILE__,
         __LINE__);
  }
}
// Workgroups of the multi-step kernel (with or without the in-launch close) resident at once
// on one CU at this block size. (0 for instantiations whose batches run chained:
// multistep_pays)
template <DivMode M, class F, bool CLOSE>
int multistep_occupancy(int block) {
  int n = 0;
  if constexpr (multistep_o8<M, F>())
    MIINT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &n, reinterpret_cast<const void*>(&riemann_multistep_kernel_o8<M, F, CLOSE>), block, 0));
  else
    MIINT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &n, reinterpret_cast<const void*>(&riemann_multistep_kernel<M, F, CLOSE>), block, 0));
  return n;
}
template <DivMode M, class F>
void multistep_per_cu_t(int block, bool close, int* out) {
  if constexpr (!multistep_pays<M, F>())
    *out = 0;
  else if constexpr (!multistep_close_ok<M, F>())
    *out = close ? 0 : multistep_occupancy<M, F, false>(block);
  else
    *out = close ? multistep_occupancy<M, F, true>(block) : multistep_occupancy<M, F, false>(block);
}

// kIeee Pi4 launches take Pi4::recip_narrow when both end coordinates (the extremes: x is
// linear in the sample index) stay below kPi4NarrowMaxX in magnitude; NaN ends do not.
std::atomic<bool> g_pi4_library_division{false};  // validation switch: always Pi4Wide
std::atomic<bool> g_trig_library{false};  // validation switch: kIeee sin/cos by ocml per sample
inline bool trig_library() { return g_trig_library.load(std::memory_order_relaxed); }
inline bool pi4_narrow(const RiemannParams& p, double max_x = kPi4NarrowMaxX) {
  if (g_pi4_library_division.load(std::memory_order_relaxed)) return false;
  const double first = static_cast<double>(p.i_begin) + p.off;
  const double last = static_cast<double>(p.i_begin + (p.n > 0 ? p.n - 1 : 0)) + p.off;
  return std::fabs(std::fma(first, p.h, p.a)) < max_x &&
         std::fabs(std::fma(last, p.h, p.a)) < max_x;
}

// Dispatch (integrand, dtype, division mode) to a template instantiation. Transcendental
// integrands (sin/cos) and the table ignore the division mode (no division in them).
template <template <DivMode, class> class Op, class... A>
void dispatch(const RiemannParams& p, DType dtype, DivMode m, A&&... a) {
  const Integrand f = static_cast<Integrand>(p.integrand);
  if (dtype == DType::kF32Acc32) {
    MIINT_CHECK(f == Integrand::kPi4, "fp32 accumulation (fp32acc) is implemented for pi4 only");
    if (m == DivMode::kSeries) Op<DivMode::kSeries, Pi4F32Acc32>::run(a...);
    else if (pi4_narrow(p, kPi4F32NarrowMaxX)) Op<DivMode::kIeee, Pi4F32Acc32>::run(a...);
    else fail("fp32acc: coordinates beyond 2^49 need the wide division (use fp32)", __FILE__,
              __LINE__);
    return;
  }
  if (dtype == DType::kF32) {
    const bool ser = m == DivMode::kSeries;
    switch (f) {
      case Integrand::kPi4:
        if (ser) Op<DivMode::kSeries, Pi4F32>::run(a...);
        else if (pi4_narrow(p, kPi4F32NarrowMaxX)) Op<DivMode::kIeee, Pi4F32>::run(a...);
        else Op<DivMode::kIeee, Pi4F32Wide>::run(a...);
        return;
      case Integrand::kSin:
        if (ser) Op<DivMode::kSeries, SinF32>::run(a...);
        else Op<DivMode::kIeee, SinF32>::run(a...);
        return;
      case Integrand::kTrainVel:
        if (ser) Op<DivMode::kSeries, TrainVelF32>::run(a...);
        else Op<DivMode::kIeee, TrainVelF32>::run(a...);
        return;
      case Integrand::kTable:
        if (ser) Op<DivMode::kSeries, TableF32>::run(a...);
        else Op<DivMode::kIeee, TableF32>::run(a...);
        return;
      case Integrand::kPoly:  // buckets as fp64
        if (ser && p.ncoef <= 4) Op<DivMode::kSeries, PolyF32<4>>::run(a...);
        else if (ser && p.ncoef <= 6) Op<DivMode::kSeries, PolyF32<6>>::run(a...);
        else if (ser && p.ncoef == 7) Op<DivMode::kSeries, PolyF32<7>>::run(a...);
        else if (ser && p.ncoef <= 8) Op<DivMode::kSeries, PolyF32<8>>::run(a...);
        else if (p.ncoef <= 4) Op<DivMode::kIeee, PolyF32<4>>::run(a...);
        else if (p.ncoef <= 8) Op<DivMode::kIeee, PolyF32<8>>::run(a...);
        else Op<DivMode::kIeee, PolyF32<16>>::run(a...);
        return;
    }
    fail("unknown integrand", __FILE__, __LINE__);
  }
  switch (f) {
    case Integrand::kPi4:
      if (m == DivMode::kSeries) Op<DivMode::kSeries, Pi4>::run(a...);
      else if (m == DivMode::kSeriesExact) Op<DivMode::kSeriesExact, Pi4>::run(a...);
      else if (m == DivMode::kSeriesDirect) Op<DivMode::kSeriesDirect, Pi4>::run(a...);
      else if (pi4_narrow(p)) Op<DivMode::kIeee, Pi4>::run(a...);
      else Op<DivMode::kIeee, Pi4Wide>::run(a...);
      return;
    case Integrand::kSin:
      if (m == DivMode::kSeries) Op<DivMode::kSeries, Sin>::run(a...);
      else if (trig_library()) Op<DivMode::kIeee, SinLib>::run(a...);
      else Op<DivMode::kIeee, Sin>::run(a...);
      return;
    case Integrand::kPoly:  // coefficient bucket (zero-padded): series 4, 6, 7, 8; Horner 4, 8, 16
      // (degree 5 and 6 get exact buckets: a padded degree-7 pair costs 11 VALU instead of 10)
      if (m == DivMode::kSeries && p.ncoef <= 4) Op<DivMode::kSeries, Poly<4>>::run(a...);
      else if (m == DivMode::kSeries && p.ncoef <= 6) Op<DivMode::kSeries, Poly<6>>::run(a...);
      else if (m == DivMode::kSeries && p.ncoef == 7) Op<DivMode::kSeries, Poly<7>>::run(a...);
      else if (m == DivMode::kSeries && p.ncoef <= 8) Op<DivMode::kSeries, Poly<8>>::run(a...);
      else if (p.ncoef <= 4) Op<DivMode::kIeee, Poly<4>>::run(a...);
      else if (p.ncoef <= 8) Op<DivMode::kIeee, Poly<8>>::run(a...);
      else Op<DivMode::kIeee, Poly<16>>::run(a...);
      return;
    case Integrand::kTrainVel:
      if (m == DivMode::kSeries) Op<DivMode::kSeries, TrainVel>::run(a...);
      else if (trig_library()) Op<DivMode::kIeee, TrainVelLib>::run(a...);
      else Op<DivMode::kIeee, TrainVel>::run(a...);
      return;
    case Integrand::kTable:
      if (m == DivMode::kSeries) Op<DivMode::kSeries, Table>::run(a...);
      else Op<DivMode::kIeee, Table>::run(a...);
      return;
  }
  fail("unknown integrand", __FILE__, __LINE__);
}

template <DivMode M, class F> struct PartialsOp {
  template <class... A> static void run(A... a) { launch_partials_t<M, F>(a...); }
};
template <DivMode M, class F> struct FusedOp {
  template <class... A> static void run(A... a) { launch_fused_t<M, F>(a...); }
};
template <DivMode M, class F> struct ChainedOp {
  template <class... A> static void run(A... a) { launch_chained_t<M, F>(a...); }
};
template <DivMode M, class F> struct MultiStepOp {
  template <class... A> static void run(A... a) { launch_multistep_t<M, F>(a...); }
};
template <DivMode M, class F> struct MultiStepOccOp {
  static void run(int block, bool close, int* out) { multistep_per_cu_t<M, F>(block, close, out); }
};
template <DivMode M, class F> struct TileLenOp {
  static void run(int* out) { *out = F::template tile_len<M>(); }
};
template <DivMode M, class F> struct PointsOp {
  static void run(const RiemannParams& p, const double* table, int table_n, double* out,
                  hipStream_t stream) {
    constexpr int T = F::template tile_len<M>();
    const uint64_t ntile = (p.n + T - 1) / T;
    const int grid = static_cast<int>((ntile + B - 1) / B);
    point_values_kernel<M, F><<<grid, B, 0, stream>>>(p, table, table_n, out);
  }
};

}  // namespace

// ============================================================================ host side
bool riemann_block_ok(int block) {
  return block == 64 || block == 128 || block == 256 || block == 512 || block == 1024;
}

LaunchShape default_riemann_shape(int num_cus, int waves_per_cu, int block) {
  MIINT_CHECK(riemann_block_ok(block), "unsupported Riemann block size");
  const int waves_per_block = block / kWave;
  int blocks = (num_cus * waves_per_cu) / waves_per_block;
  if (blocks < 1) blocks = 1;
  return {blocks, block};
}

double integrand_scale(Integrand f) { return f == Integrand::kPi4 ? Pi4::kScale : 1.0; }

static void check_shape(LaunchShape s) {
  MIINT_CHECK(riemann_block_ok(s.block),
              "riemann kernels run 64-, 128-, 256-, 512- or 1024-thread workgroups (got " +
                  std::to_string(s.block) + ")");
  MIINT_CHECK(s.grid >= 1 && s.grid <= (1 << 20), "grid out of range");
}

static void check_params(const RiemannParams& p, const double* table, int table_n) {
  const int f = p.integrand;
  MIINT_CHECK(f >= 0 && f <= static_cast<int>(Integrand::kTable), "unknown integrand");
  if (static_cast<Integrand>(f) == Integrand::kTable) {
    MIINT_CHECK(table != nullptr, "table integrand needs a device table");
    MIINT_CHECK(table_n >= 2 && table_n <= kMaxTable, "table size must be in [2, 2048]");
  }
  if (static_cast<Integrand>(f) == Integrand::kPoly)
    MIINT_CHECK(p.ncoef >= 1 && p.ncoef <= kMaxPolyCoeffs, "poly needs 1..16 coefficients");
  if (static_cast<Integrand>(f) == Integrand::kTrainVel)
    MIINT_CHECK(p.p0 != 0.0, "train integrand needs ts != 0");
  MIINT_CHECK(p.i_begin + p.n < (uint64_t(1) << 52), "sample index must stay below 2^52");
}

static DivMode effective_div(const RiemannParams& p, DivMode div, DType dtype) {
  return miint::effective_div(div, p.h, static_cast<Integrand>(p.integrand), dtype, p.ncoef);
}

// Host-side constants of the angle-addition series (long double; AngleSeries in
// integrands.hpp): delta = h for sin, h / ts for the train velocity.
static RiemannParams prepared(const RiemannParams& p, DivMode eff) {
  RiemannParams q = p;
  const Integrand f = static_cast<Integrand>(p.integrand);
  if (f == Integrand::kPoly && eff == DivMode::kSeries) {  // c_i h^i for the Taylor shift
    long double hp = 1.0L;
    for (int i = 0; i < kMaxPolyCoeffs; ++i) {
      q.coef_h[i] = i < p.ncoef ? static_cast<double>(static_cast<long double>(p.coef[i]) * hp)
                                : 0.0;
      hp *= static_cast<long double>(p.h);
    }
  }
  if ((f == Integrand::kSin || f == Integrand::kTrainVel) && eff == DivMode::kSeries) {
    // (the fp32 functors read the same table, rounded to fp32 on the device)
    const long double delta =
        f == Integrand::kSin ? static_cast<long double>(p.h)
                             : static_cast<long double>(p.h) / static_cast<long double>(p.p0);
    for (int j = 0; j < AngleSeries<12>::kPairs; ++j) {
      const long double k = j + 0.5L;
      q.trig[j] = static_cast<double>(cosl(k * delta));
      q.trig[AngleSeries<12>::kPairs + j] = static_cast<double>(sinl(k * delta));
    }
    for (int i = 0; i < AngleSeries<12>::kSubs / 2; ++i) {
      const long double c0 = AngleSeries<12>::kSub * (i + 0.5L);
      q.trig[2 * AngleSeries<12>::kPairs + 2 * i] = static_cast<double>(cosl(c0 * delta));
      q.trig[2 * AngleSeries<12>::kPairs + 2 * i + 1] = static_cast<double>(sinl(c0 * delta));
    }
    for (int i = 0; i < kSinTrig; ++i) q.trig32[i] = static_cast<float>(q.trig[i]);
  }
  return q;
}

int riemann_tile_len(const RiemannParams& p, DType dtype, DivMode div) {
  int t = 0;
  dispatch<TileLenOp>(p, dtype, effective_div(p, div, dtype), &t);
  return t;
}

void launch_riemann_partials(const RiemannParams& p, DType dtype, DivMode div, LaunchShape shape,
                             const double* table, int table_n, double* partials,
                             hipStream_t stream) {
  check_shape(shape);
  check_params(p, table, table_n);
  const DivMode eff = effective_div(p, div, dtype);
  dispatch<PartialsOp>(p, dtype, eff, prepared(p, eff), shape, table, table_n, partials, stream);
  MIINT_HIP(hipGetLastError());
}

void launch_finalize(const double* partials, int n, double scale, double* out,
                     hipStream_t stream, int block) {
  MIINT_CHECK(n >= 1, "finalize needs at least one partial");
  MIINT_CHECK(riemann_block_ok(block), "unsupported finalize block size");
  finalize_kernel<<<1, block, 0, stream>>>(partials, n, scale, out);
  MIINT_HIP(hipGetLastError());
}

void launch_riemann_fused(const RiemannParams& p, DType dtype, DivMode div, LaunchShape shape,
                          const double* table, int table_n, double* partials,
                          unsigned int* ticket, double scale, double* out, hipStream_t stream) {
  check_shape(shape);
  check_params(p, table, table_n);
  const DivMode eff = effective_div(p, div, dtype);
  dispatch<FusedOp>(p, dtype, eff, prepared(p, eff), shape, table, table_n, partials, ticket,
                    scale, out, stream);
  MIINT_HIP(hipGetLastError());
}

void launch_riemann_chained(const RiemannParams& p, DType dtype, DivMode div, LaunchShape shape,
                            const double* table, int table_n, double* partials,
                            const double* prev, int nprev, double scale, double* out_prev,
                            hipStream_t stream) {
  check_shape(shape);
  check_params(p, table, table_n);
  MIINT_CHECK(prev == nullptr || (nprev == shape.grid && out_prev != nullptr),
              "chained finalize: previous partials must come from the same grid");
  const DivMode eff = effective_div(p, div, dtype);
  dispatch<ChainedOp>(p, dtype, eff, prepared(p, eff), shape, table, table_n, partials, prev,
                      nprev, scale, out_prev, stream);
  MIINT_HIP(hipGetLastError());
}

int riemann_multistep_grid(const RiemannParams& p, DType dtype, DivMode div, int block,
                          int num_cus, bool close) {
  MIINT_CHECK(riemann_block_ok(block), "unsupported Riemann block size");
  int per_cu = 0;
  dispatch<MultiStepOccOp>(p, dtype, effective_div(p, div, dtype), block, close, &per_cu);
  return per_cu * num_cus;  // 0: this instantiation runs chained batches
}

void launch_riemann_multistep(const RiemannParams& p, DType dtype, DivMode div,
                              LaunchShape shape, const double* table, int table_n,
                              double* partials, int steps, double scale, double* out,
                              hipStream_t stream, unsigned int* ticket, bool close_kernel) {
  check_shape(shape);
  check_params(p, table, table_n);
  MIINT_CHECK(steps >= 1 && steps <= kMaxMultiSteps, "multi-step launch: 1..64 steps");
  MIINT_CHECK(partials != nullptr && out != nullptr, "multi-step launch needs partials and results");
  const DivMode eff = effective_div(p, div, dtype);
  // rotation: the blocks owning one tile round more than the rest (lane_sum: the first
  // `heavy`) move by `heavy` blocks a step, so each workgroup gets its share of them
  int tl = 0;
  dispatch<TileLenOp>(p, dtype, eff, &tl);
  const uint64_t lanes = static_cast<uint64_t>(shape.grid) * static_cast<uint64_t>(shape.block);
  const uint64_t extra = (p.n / static_cast<uint64_t>(tl)) % lanes;
  const unsigned heavy = static_cast<unsigned>((extra + shape.block - 1) / shape.block);
  const unsigned rot = heavy % static_cast<unsigned>(shape.grid);
  dispatch<MultiStepOp>(p, dtype, eff, prepared(p, eff), shape, table, table_n, partials, steps,
                        rot, ticket, scale, out, stream);
  MIINT_HIP(hipGetLastError());
  if (ticket || !close_kernel) return;  // closed inside the launch, or by the caller
  launch_multistep_close(partials, shape.grid, steps, scale, out, shape.block, stream);
}

void launch_multistep_close(const double* partials, int grid, int steps, double scale,
                            double* out, int block, hipStream_t stream) {
  MIINT_CHECK(steps >= 1 && steps <= kMaxMultiSteps && grid >= 1 && riemann_block_ok(block),
              "multi-step close: 1..64 steps, a Riemann block size");
  multistep_close_kernel<<<steps, block, 0, stream>>>(partials, grid, scale, out);
  MIINT_HIP(hipGetLastError());
}

void launch_riemann_point_values(const RiemannParams& p, DivMode div, const double* table,
                                 int table_n, double* out, hipStream_t stream) {
  check_params(p, table, table_n);
  MIINT_CHECK(p.n >= 1, "empty range");
  const DivMode eff = effective_div(p, div, DType::kF64);
  dispatch<PointsOp>(p, DType::kF64, eff, prepared(p, eff), table, table_n, out, stream);
  MIINT_HIP(hipGetLastError());
}

void set_pi4_library_division(bool on) { g_pi4_library_division.store(on); }
void set_trig_library(bool on) { g_trig_library.store(on); }

void launch_pi4_recip_narrow(const double* d, uint64_t n, double* out, hipStream_t stream) {
  if (n == 0) return;
  const uint64_t blocks = (n + B - 1) / B;
  const int grid = static_cast<int>(blocks < 8192 ? blocks : 8192);
  recip_narrow_kernel<<<grid, B, 0, stream>>>(d, n, out);
  MIINT_HIP(hipGetLastError());
}

void launch_pi4_recip_narrow_f32(const float* d, uint64_t n, float* out, hipStream_t stream) {
  if (n == 0) return;
  const uint64_t blocks = (n + B - 1) / B;
  const int grid = static_cast<int>(blocks < 8192 ? blocks : 8192);
  recip_narrow_f32_kernel<<<grid, B, 0, stream>>>(d, n, out);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
