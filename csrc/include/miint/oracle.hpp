// Host-side oracles, fixtures and reference-parity emulation.
//
// The reference has no tests; its only checks are eyeballing printed values.
// This module provides the numbers every test and CLI self-check compares against:
//   * the 1801-sample velocity profile: bit-exact data
//     (profile_data.cpp, sha256-pinned), plus a generator of the same profile from its
//     7-phase jerk-limited definition (within 1.1e-13 of the data) as a cross-check;
//   * serial long-double Riemann sums and analytic integrals;
//   * exact emulations of the reference programs' partition arithmetic, bugs included
//     (SURVEY §2.7 B5/B10/B13), behind --parity switches in the CLIs.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "miint/common.hpp"

namespace miint {
namespace oracle {

// ------------------------------------------------------------------ velocity profile
constexpr int kProfileLen = 1801;        // ex4vel.h:5 "200 lines of 9 numbers + 1"
constexpr int kProfileSeconds = 1800;
constexpr int kStepsPerSec = 10000;      // cintegrate.cu:19, 4main.c:26
constexpr double kJerk = 0.002904762;    // m/s^3 per 1-s step of the profile

// DefaultProfile (ex4vel.h:10-210), bit-exact: what every kernel, plan and oracle uses.
const std::vector<double>& profile_table();
// The same profile generated from its definition: v[0]=0, v[i+1]=v[i]+a_i with a_i the
// jerk-limited acceleration (ramp 100 s, hold 200 s, ramp-down 100 s, cruise 1000 s,
// mirrored braking), rounded to 15 significant digits (ex4vel.h:1-5 "Excel ... 15 digits").
// Within 1.1e-13 of profile_table(); kept as an independent check of the data.
const std::vector<double>& generated_profile_table();

// A velocity profile from a text/CSV file (the reference's table was "Auto-generated from
// Excel CSV", ex4vel.h:1-5): numbers separated by commas, whitespace or newlines, one sample
// per second; '#' starts a comment line. At least 2 finite values, else an error.
std::vector<double> load_profile(const std::string& path);
// Exact integral over [a, b] (inside [0, len - 1]) of the table's piecewise-linear
// interpolant at unit spacing.
double table_integral(const std::vector<double>& table, double a, double b);
// Linear interpolation of a 1-s-spaced table at t, segment index clamped to the table.
double interp(const std::vector<double>& table, double t);

// Exact integral of the piecewise-linear interpolant over [0, 1800] (trapezoid, dt=1):
// 122000.004000.
double profile_exact_integral();

// ------------------------------------------------------------------ analytic values
double analytic(Integrand f, double a, double b, const std::vector<double>& coef = {},
                double p0 = 0.0, double p1 = 0.0);

// Serial reference Riemann sum in long double with Kahan compensation.
long double riemann_serial(Integrand f, double a, double b, uint64_t n, Rule rule,
                           const std::vector<double>& coef = {}, double p0 = 0.0,
                           double p1 = 0.0, const std::vector<double>* table = nullptr);

// Analytic-train constants (riemann.cpp:7-9).
constexpr double kTrainTs = 286.4788975;
constexpr double kTrainAs = 0.2365890;
constexpr double kTrainVs = 67.7777777;
double train_distance(double t);  // dis_function (riemann.cpp:113-116)

// ------------------------------------------------------------------ parity emulation
// riemann.cpp master/worker: P ranks -> P-1 workers, worker w integrates
// [w*R/W, (w+1)*R/W) with (int)(n/W) samples sequentially, root sums in rank order.
// P == 1 -> 0. Sequential fp64, like the reference.
double riemann_mpi_parity(int comm_size, double n, double range = 3.14159265358979323846);

// cintegrate.cu cuda_test with SP x SM threads: thread r sums interp(i*dt) for
// i in [r*floor(1800/W)*1e4, (r+1)*floor(1800/W)*1e4) sequentially; host sums threads
// in order. SP=32, SM=2 -> 121999.800663 (coverage truncation B5).
double cintegrate_parity(int sp, int sm);

// 4main.c with P ranks: per-rank private InterpProfile fill by seconds, scan partition by
// elements with the residual never scanned, root carry fix-up; returns the printed
// "Total distance traveled" (default_sum[T-2]/1e4) and the phase-2 sum-of-sums total.
struct TrainScanParity {
  double distance;      // what 4main prints
  double sum_of_sums;   // default_sum_of_sums[T-1] on root after phase 2 (never printed)
};
TrainScanParity trainscan_parity(int comm_size);
// The reference's faccel (4main.c:262-269) bit-for-bit: no clamping, no FMA.
double faccel_ref(const std::vector<double>& table, double time);

}  // namespace oracle
}  // namespace miint
