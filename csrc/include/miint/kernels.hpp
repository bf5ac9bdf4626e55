// Host-side launch API for every miint HIP kernel (gfx950 only).
//
// All launchers are asynchronous on the given stream, allocate nothing and never
// synchronise, so they can be captured into a hipGraph (cdna_hip_programming.md §6 G9).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

#include "miint/common.hpp"

namespace miint {

// kF32Acc32: the fp32 sample path with fp32 accumulation down to the workgroup partial
// (lane sums, v_add_f32_dpp wave reduction, LDS block step; the partials meet in fp64) —
// the all-fp32 reduction BASELINE #4 names, measured against kF32's fp64 fold. 4/(1+x^2)
// only.
enum class DType : int { kF64 = 0, kF32 = 1, kF32Acc32 = 2 };
inline bool is_fp32(DType t) { return t == DType::kF32 || t == DType::kF32Acc32; }

// Tile (unroll) size of the Riemann kernels: U consecutive samples per lane per step.
constexpr int kRiemannTile = 32;     // default samples per lane tile (Pi4 series: 64)
constexpr int kRiemannBlock = 256;
constexpr int kSeriesHalfSpan = 192;    // max |sample offset| from an fp64 Pi4 series seed, in steps
constexpr int kSeriesHalfSpanF32 = 96;  // the same for the fp32 Pi4 series tiles

constexpr int kDirectHalfSpan = 16;  // the same for kSeriesDirect's 32-sample tiles

// True when the fp64 Pi4 series reciprocal is exact to fp64 for this h (see integrands.hpp).
inline bool series_ok(double h) { return kSeriesHalfSpan * (h < 0 ? -h : h) <= 2e-6; }
inline bool series_ok_f32(double h) { return kSeriesHalfSpanF32 * (h < 0 ? -h : h) <= 2e-6; }
inline bool direct_ok(double h) { return kDirectHalfSpan * (h < 0 ? -h : h) <= 2e-6; }

// Division mode actually used for step h: the 384-sample series tiles need N >= 9.6e7 on
// [0, 1]; a coarser step still fits the 32-sample kSeriesDirect tiles down to N = 8e6
// (5 VALU per sample against ~10 for IEEE division); coarser steps use IEEE division.
inline DivMode effective_div(DivMode d, double h) {
  if (d == DivMode::kIeee) return d;
  if ((d == DivMode::kSeries || d == DivMode::kSeriesExact) && series_ok(h)) return d;
  return direct_ok(h) ? DivMode::kSeriesDirect : DivMode::kIeee;
}
// Per integrand: the sin / train-velocity series path (angle addition from a per-tile sincos
// seed) and the table's segment-line tiles are exact for any h, so only the series/ieee
// choice applies (kSeriesExact, the exact-grade request, is their series path); integrands
// without a series path run kIeee.
inline bool series_request(DivMode d) { return d == DivMode::kSeries || d == DivMode::kSeriesExact; }
inline DivMode effective_div(DivMode d, double h, Integrand f) {
  if (f == Integrand::kSin || f == Integrand::kTrainVel || f == Integrand::kTable)
    return series_request(d) ? DivMode::kSeries : DivMode::kIeee;
  if (f != Integrand::kPi4) return DivMode::kIeee;
  return effective_div(d, h);
}

constexpr int kPolySeriesMaxCoeffs = 8;  // polynomials up to degree 7 have a series path

// With the dtype (the fp32 paths: pi4's 192-sample first-order tiles where series_ok_f32, and
// the packed-fp32 forms of the other integrands' series tiles) and the polynomial's
// coefficient count (Taylor-pair tiles for up
// to kPolySeriesMaxCoeffs coefficients, exact for any h; Horner per sample otherwise).
inline DivMode effective_div(DivMode d, double h, Integrand f, DType t, int ncoef = 0) {
  if (is_fp32(t)) {  // fp32: one series form per integrand (integrands_f32.hpp)
    if (d == DivMode::kIeee) return DivMode::kIeee;
    if (f == Integrand::kPi4) return series_ok_f32(h) ? DivMode::kSeries : DivMode::kIeee;
    if (f == Integrand::kPoly)
      return (ncoef >= 1 && ncoef <= kPolySeriesMaxCoeffs) ? DivMode::kSeries : DivMode::kIeee;
    return DivMode::kSeries;  // sin, train velocity, table: exact for any h
  }
  if (f == Integrand::kPoly)  // the Taylor-pair tiles are exact-grade: kSeriesExact runs them
    return (series_request(d) && ncoef >= 1 && ncoef <= kPolySeriesMaxCoeffs)
               ? DivMode::kSeries
               : DivMode::kIeee;
  return effective_div(d, h, f);
}

struct LaunchShape {
  int grid;   // workgroups
  int block;  // threads per workgroup
};

// Block sizes the Riemann kernels run (--block): 64, 128, 256 (default), 512, 1024.
bool riemann_block_ok(int block);
// Default grid: enough workgroups of `block` threads to hold `waves_per_cu` waves on every CU.
LaunchShape default_riemann_shape(int num_cus, int waves_per_cu = 32, int block = kRiemannBlock);

// Riemann partial sums: writes one fp64 partial per workgroup into partials[0..grid).
// Partials are *unscaled* sums of f; multiply by h * integrand scale at finalize.
// `table` (device, `table_n` doubles) is used only for Integrand::kTable.
void launch_riemann_partials(const RiemannParams& p, DType dtype, DivMode div,
                             LaunchShape shape, const double* table, int table_n,
                             double* partials, hipStream_t stream);

// out[0] = scale * sum(partials[0..n)) in a fixed order (bitwise reproducible): one
// workgroup of `block` threads, the same order as a fused launch at that block size.
void launch_finalize(const double* partials, int n, double scale, double* out,
                     hipStream_t stream, int block = kRiemannBlock);

// Fill `count` doubles with the write-once slots' unset pattern (handoff.hpp).
constexpr unsigned kUnsetSlotWord = 0xFFFAFFFAu;
void fill_unset_slots(double* p, size_t count, hipStream_t stream);

// Ticket of the one-launch reduction: kTicketGroups group counters and one top counter,
// each on its own 256-byte line (kTicketWords unsigned words in all). A single counter
// serialised 2048 same-address atomics at the end of every launch (~14 us at N = 1e8).
constexpr int kTicketGroups = 16;
constexpr int kTicketStride = 64;  // words between counters (256 B)
constexpr int kTicketWords = (kTicketGroups + 1) * kTicketStride;

// One-launch variant: partials + last-workgroup ticket reduction (write-once slots,
// handoff.hpp; cdna_hip_programming.md §6 G16). `ticket` (kTicketWords words) must be zero
// and `partials` (grid doubles) filled with the unset pattern (fill_unset_slots) before the
// first launch; the last workgroup re-arms both.
void launch_riemann_fused(const RiemannParams& p, DType dtype, DivMode div, LaunchShape shape,
                          const double* table, int table_n, double* partials,
                          unsigned int* ticket, double scale, double* out, hipStream_t stream);

// Batched steps without the ticket: writes this step's partials into partials[0..grid) and,
// if prev != nullptr, its last workgroup first stores scale * (index-ordered sum of
// prev[0..nprev)) into out_prev[0] (the previous step's result; nprev == grid). Close a
// batch with launch_finalize on the last step's partials. Same sums, bit for bit, as the
// fused and two-kernel paths.
void launch_riemann_chained(const RiemannParams& p, DType dtype, DivMode div, LaunchShape shape,
                            const double* table, int table_n, double* partials,
                            const double* prev, int nprev, double scale, double* out_prev,
                            hipStream_t stream);

// K = `steps` complete integrations in one persistent launch, closed by one K-workgroup
// kernel (riemann.hip "multi-step"): out[s] = step s's scaled sum, bitwise the fused /
// chained / two-kernel value at the same grid. `partials` holds steps x grid doubles. The
// grid should be resident as a whole: at most riemann_multistep_grid(...) workgroups (0 for
// the instantiations that keep chained batches).
// ticket != nullptr (kTicketWords words, zero before the first launch; re-armed by the
// kernel): no closing kernel — the launch's last arrivals close the batch themselves
// (handoff.hpp close_batch_in_launch), bitwise the same values; its residency is
// riemann_multistep_grid(..., close = true).
// 1 <= steps <= kMaxMultiSteps.
constexpr int kMaxMultiSteps = 64;
int riemann_multistep_grid(const RiemannParams& p, DType dtype, DivMode div, int block,
                           int num_cus, bool close = false);
void launch_riemann_multistep(const RiemannParams& p, DType dtype, DivMode div,
                              LaunchShape shape, const double* table, int table_n,
                              double* partials, int steps, double scale, double* out,
                              hipStream_t stream, unsigned int* ticket = nullptr,
                              bool close_kernel = true);
// The closing kernel of a multi-step launch on its own (launch_riemann_multistep with
// close_kernel = false, e.g. to time the two apart): out[s] = scale * step s's sum.
void launch_multistep_close(const double* partials, int grid, int steps, double scale,
                            double* out, int block, hipStream_t stream);

// Debug/validation: write every sample's f value (as the hot tile path computes it) to
// `out[0..p.n)`; fp64 only. Used by the per-point accuracy tests of the series division.
void launch_riemann_point_values(const RiemannParams& p, DivMode div, const double* table,
                                 int table_n, double* out, hipStream_t stream);

// Validation: out[i] = the kIeee Pi4 tiles' reciprocal of d[i] (Pi4::recip_narrow; equal to
// IEEE 1.0 / d[i] for 1 <= d[i] <= 2^500).
void launch_pi4_recip_narrow(const double* d, uint64_t n, double* out, hipStream_t stream);
// The same for the fp32 kIeee tiles (Pi4F32::recip_narrow; IEEE 1.0f / d for 1 <= d <= 2^100).
void launch_pi4_recip_narrow_f32(const float* d, uint64_t n, float* out, hipStream_t stream);
// Validation: when on, kIeee Pi4 launches run the library division everywhere (Pi4Wide,
// Pi4F32Wide), so tests can check that the two give bitwise the same sums.
void set_pi4_library_division(bool on);
// Validation switch: kIeee sin (Sin) and cos (TrainVel) by ocml per sample instead of the
// fast per-sample path (fast_trig.hpp). Process-wide; tests only.
void set_trig_library(bool on);
// Validation switch: every kernel that stages a WINDOW of a table in LDS (train-scan samplers,
// interp_fill chunks, the 2-D row stream's footprint tile) first fills its LDS buffer with
// NaN (the 2-D stream: every tile slot outside the computed footprint), so a read past the
// staged window yields NaN instead of a stale-but-finite word. Per device (the current one),
// process-wide; tests only.
void set_lds_poison(bool on);
void set_lds_poison_trainscan(bool on);  // (per kernel file; set_lds_poison sets all)
void set_lds_poison_table(bool on);

// Samples per lane tile of the kernel that launch_riemann_* would run for these arguments
// (32; 64 or 128 on the series paths): host-side grid sizing.
int riemann_tile_len(const RiemannParams& p, DType dtype, DivMode div);

// Integrand scale factor (4 for Pi4, 1 otherwise).
double integrand_scale(Integrand f);

// ---------------------------------------------------------------- reductions / tables
// out[0] = scale * sum(x[0..n)) — vectorised HBM-bound two-pass sum (fixed order).
// `partials` needs default_reduce_grid() doubles.
int default_reduce_grid(int num_cus);
void launch_sum_array(const double* x, uint64_t n, double scale, double* partials, int grid,
                      double* out, hipStream_t stream);

// Materialise the interpolated profile: y[i] = interp(table, (i0 + i) * dt) for i < n.
// (cintegrate.cu:88-92 / 4main.c:82-86 fill loop, coalesced and LDS-staged here.)
void launch_interp_fill(const double* table, int table_n, double dt, uint64_t i0, uint64_t n,
                        double* y, hipStream_t stream);

// ---------------------------------------------------------------- scan (scan.hip)
// Single-pass decoupled look-back inclusive scan of fp64 (replaces 4main.c:95-221's
// gather-to-root + serial carry + broadcast). `state` needs scan_state_bytes(n) bytes and
// is re-initialised by the launcher on the stream every call. out may alias in.
// If `carry_in` is non-null its device value is added to every output (multi-GPU carry).
size_t scan_state_bytes(uint64_t n);
void launch_inclusive_scan(const double* in, double* out, uint64_t n, void* state,
                           const double* carry_in, hipStream_t stream);
// Fused: y = inclusive_scan(interp(table, (i0+i)*dt)) without materialising the fill.
void launch_interp_scan(const double* table, int table_n, double dt, uint64_t i0, uint64_t n,
                        double* out, void* state, const double* carry_in, hipStream_t stream);
// Same, but samples whose global index i0+g lies outside [win_lo, win_hi) contribute 0:
// emulates 4main.c's per-rank private fill windows (4main.c:76-86) for --parity runs.
void launch_interp_scan_window(const double* table, int table_n, double dt, uint64_t i0,
                               uint64_t n, uint64_t win_lo, uint64_t win_hi, double* out,
                               void* state, const double* carry_in, hipStream_t stream);
// Reads back the scan's spin-timeout word (non-zero = a look-back gave up; never expected).
unsigned scan_timeout_flag(const void* state, hipStream_t stream);
// x[i] += carry[0] for i < n (fix-up after a multi-GPU carry exchange).
void launch_add_carry(double* x, uint64_t n, const double* carry, hipStream_t stream);

// ---------------------------------------------------------------- 2-D table (table2d.hip)
// Integrate the bilinear interpolant of a row-major ny x nx fp64 table spanning
// [0, X] x [0, Y] with a midpoint rule on gx x gy points, rows [row0, row1) of the sample
// grid only (multi-GPU row split). Writes one partial per workgroup.
struct Table2DParams {
  const double* table;
  int nx, ny;        // table dims (entries)
  double X, Y;       // physical extents
  int gx, gy;        // sample grid
  int row0, row1;    // sample rows owned by this launch
  int min_wg = 0;    // row stream: fewest workgroups to aim for (0 = 512)
};
int table2d_grid(const Table2DParams& p);
// Which kernel a launch runs: "stream" (LDS footprint + row streaming, fine grids) or
// "tile" (coarse grids, table read from global memory).
const char* table2d_path(const Table2DParams& p);
// The launch shape table2d_* pick (host only; tests check the footprint bound against it):
// row stream or tile, rows per wave, staged tile rows (kSH or the short tile), tile width,
// grid, and for the tile kernel its square size.
struct Table2DShapeInfo {
  bool stream;
  int rows_per_wave, tile_rows, tile_cols, grid_x, grid_y, tile;
};
Table2DShapeInfo table2d_shape_info(const Table2DParams& p);
// Multi-step row stream: `steps` integrations in one launch, then one closing kernel:
// outs[s] = integration s, bitwise the chained / fused value. `partials` holds steps x
// table2d_grid(p) doubles. Only for launches table2d_multistep_ok accepts (the row-stream
// shape; residency is not required: no workgroup waits on another).
// Step phases: the launch holds `phases` workgroups per row-stream block, workgroup phase f
// running the steps s = f, f + phases, ... of its block — steps are independent, and a block
// step is latency-bound (staging, a short row loop, the block reduction) at 2 waves per SIMD,
// so several steps of one block in flight on different workgroups overlap those latencies.
// Every partial is still one workgroup's, computed as in the one-phase launch: bitwise the
// same values. 0 = auto: kT2AutoPhases (<= steps) — past residency the later phases'
// workgroups start as earlier ones finish, and 16 phases measured fastest or level on every
// shape (profiles/r4/t2d_phases_explicit.jsonl, t2d_variant_ab.jsonl, t2d_shape_sweep.jsonl) —
// doubled while the launch would hold fewer than kT2AutoWorkgroups workgroups (small row
// slices at the long replays of round 5, profiles/r5/t2d/n_t2d_steps.jsonl).
constexpr int kT2AutoPhases = 16;  // auto (at least)
constexpr long kT2AutoWorkgroups = 4096;  // auto: phases double while nb x phases is below
constexpr int kT2MaxPhases = 32;  // an explicit request (32: one step per workgroup)
constexpr int kT2MaxReplaySteps = 1024;  // launch_table2d_multistep's step limit
bool table2d_multistep_ok(const Table2DParams& p, int num_cus);
// Multi-step workgroups resident per CU (hipOccupancy; 0 for a shape without the row stream).
int table2d_multistep_resident(const Table2DParams& p);
int table2d_multistep_phases(const Table2DParams& p, int num_cus, int steps, int want = 0);
void launch_table2d_multistep(const Table2DParams& p, double* partials, int steps, double* outs,
                              hipStream_t stream, int phases = 1);
void launch_table2d_partials(const Table2DParams& p, double* partials, hipStream_t stream);
// One launch: partials + last-workgroup reduction into out[0] (ticket: kTicketWords words,
// zero before the first launch; partials: table2d_grid(p) doubles filled with the unset
// pattern (fill_unset_slots); both re-armed by the kernel).
void launch_table2d_fused(const Table2DParams& p, double* partials, unsigned* ticket,
                          double* out, hipStream_t stream);
// Batches of integrations of the same field: launch j writes its table2d_grid(p) partials
// into `partials` (one half of a double buffer) and, if prev != nullptr, its workgroup 0
// first sums launch j-1's partials (the other half, same p) into *prev_out; the batch's last
// partials are closed by launch_table2d_finalize. Values are bitwise those of the fused
// launch.
void launch_table2d_chained(const Table2DParams& p, double* partials, const double* prev,
                            double* prev_out, hipStream_t stream);
void launch_table2d_finalize(const double* partials, int n, double* out, hipStream_t stream);
void launch_outer_product(const double* v, int n, double* table, hipStream_t stream);

}  // namespace miint
