// Host oracles, generated fixtures and parity emulation (see miint/oracle.hpp).
#include "miint/oracle.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

namespace miint {
namespace oracle {

namespace {

double round15(double x) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.15g", x);
  return std::strtod(buf, nullptr);
}

// Jerk-step multiplier k_i for the acceleration of second i (a_i = k_i * kJerk), the
// discrete form of the 7-phase profile: +jerk 100 s, hold 200 s, -jerk 99 s, cruise,
// -jerk 99 s, hold, +jerk 99 s, rest.
int accel_steps(int i) {
  if (i < 100) return i + 1;
  if (i < 300) return 100;
  if (i < 399) return 399 - i;
  if (i < 1400) return 0;
  if (i < 1499) return -(i - 1399);
  if (i < 1700) return -100;
  if (i < 1799) return -(1799 - i);
  return 0;
}

std::vector<double> make_profile() {
  std::vector<double> v(kProfileLen);
  double vel = 0.0, acc = 0.0;
  int kprev = 0;
  v[0] = 0.0;
  for (int i = 0; i < kProfileSeconds; ++i) {
    const int k = accel_steps(i);
    acc = acc + static_cast<double>(k - kprev) * kJerk;  // spreadsheet-style running sums
    kprev = k;
    vel = vel + acc;
    v[i + 1] = vel;
  }
  for (double& x : v) x = round15(x);
  return v;
}

}  // namespace

extern const double kProfileData[kProfileLen];  // profile_data.cpp (bit-exact ex4vel.h)

const std::vector<double>& profile_table() {
  static const std::vector<double> t(kProfileData, kProfileData + kProfileLen);
  return t;
}

const std::vector<double>& generated_profile_table() {
  static const std::vector<double> t = make_profile();
  return t;
}

std::vector<double> load_profile(const std::string& path) {
  std::ifstream in(path);
  MIINT_CHECK(in.good(), "cannot read profile " + path);
  std::vector<double> v;
  std::string line;
  int lineno = 0;
  while (std::getline(in, line)) {
    ++lineno;
    const size_t first = line.find_first_not_of(" \t\r");
    if (first == std::string::npos || line[first] == '#') continue;
    for (char& c : line)
      if (c == ',' || c == ';' || c == '\t' || c == '\r') c = ' ';
    std::istringstream ls(line);
    std::string tok;
    while (ls >> tok) {
      char* end = nullptr;
      const double x = std::strtod(tok.c_str(), &end);
      MIINT_CHECK(end && *end == '\0' && std::isfinite(x),
                  path + ":" + std::to_string(lineno) + ": not a finite number: '" + tok + "'");
      v.push_back(x);
    }
  }
  MIINT_CHECK(v.size() >= 2, path + ": a profile needs at least 2 samples");
  return v;
}

double table_integral(const std::vector<double>& v, double a, double b) {
  const int len = static_cast<int>(v.size());
  auto prim = [&](double t) {  // integral of the interpolant from 0 to t (t within the table)
    long double s = 0.0L;
    int i = 0;
    for (; i + 1 < len && i + 1 <= t; ++i) s += 0.5L * ((long double)v[i] + v[i + 1]);
    if (i + 1 < len && t > i) {
      const double fr = t - i;
      s += fr * v[i] + 0.5L * fr * fr * (v[i + 1] - v[i]);
    }
    return s;
  };
  return static_cast<double>(prim(b) - prim(a));
}

double interp(const std::vector<double>& table, double t) {
  const int nseg = static_cast<int>(table.size()) - 1;
  // segment clamped in fp64 before the conversion (a coordinate far outside the table, or
  // NaN -> segment 0, never reaches an out-of-range double -> int conversion)
  double seg = std::trunc(t);
  seg = seg > nseg - 1 ? nseg - 1 : seg;
  seg = seg >= 0.0 ? seg : 0.0;
  const int i = static_cast<int>(seg);
  const double fr = t - seg;
  return std::fma(table[i + 1] - table[i], fr, table[i]);
}

double profile_exact_integral() {
  const auto& v = profile_table();
  long double s = 0.0L;
  for (int i = 0; i + 1 < kProfileLen; ++i) s += 0.5L * (static_cast<long double>(v[i]) + v[i + 1]);
  return static_cast<double>(s);
}

double train_distance(double t) { return kTrainVs * (t - kTrainTs * std::sin(t / kTrainTs)); }

double analytic(Integrand f, double a, double b, const std::vector<double>& coef, double p0,
                double p1) {
  switch (f) {
    case Integrand::kPi4: return 4.0 * (std::atan(b) - std::atan(a));
    case Integrand::kSin: return std::cos(a) - std::cos(b);
    case Integrand::kPoly: {
      long double s = 0.0L;
      for (size_t k = 0; k < coef.size(); ++k) {
        const long double e = static_cast<long double>(k + 1);
        s += coef[k] * (std::pow(static_cast<long double>(b), e) -
                        std::pow(static_cast<long double>(a), e)) / e;
      }
      return static_cast<double>(s);
    }
    case Integrand::kTrainVel: {
      // integral of (1 - cos(t/ts)) vs = vs (t - ts sin(t/ts))
      const double ts = p0, vs = p1;
      return vs * ((b - ts * std::sin(b / ts)) - (a - ts * std::sin(a / ts)));
    }
    case Integrand::kTable:
      return table_integral(profile_table(), a, b);
  }
  return 0.0;
}

long double riemann_serial(Integrand f, double a, double b, uint64_t n, Rule rule,
                           const std::vector<double>& coef, double p0, double p1,
                           const std::vector<double>* table) {
  const long double h = (static_cast<long double>(b) - a) / n;
  const long double off = rule == Rule::kLeft ? 0.0L : (rule == Rule::kMid ? 0.5L : 1.0L);
  const std::vector<double>& tab = table ? *table : profile_table();
  long double s = 0.0L, c = 0.0L;
  for (uint64_t i = 0; i < n; ++i) {
    const long double x = a + (static_cast<long double>(i) + off) * h;
    long double y = 0.0L;
    switch (f) {
      case Integrand::kPi4: y = 4.0L / (1.0L + x * x); break;
      case Integrand::kSin: y = std::sin(x); break;
      case Integrand::kPoly: {
        for (size_t k = coef.size(); k-- > 0;) y = y * x + coef[k];
        break;
      }
      case Integrand::kTrainVel: y = (1.0L - std::cos(x / p0)) * p1; break;
      case Integrand::kTable: y = interp(tab, static_cast<double>(x)); break;
    }
    const long double yk = y - c;  // Kahan
    const long double t = s + yk;
    c = (t - s) - yk;
    s = t;
  }
  return s * h;
}

double riemann_mpi_parity(int comm_size, double n, double range) {
  const int workers = comm_size - 1;
  // the reference's `int local_n = N / W` (riemann.cpp:72): beyond INT_MAX that conversion is
  // undefined behaviour there; here it is refused instead of emulated
  MIINT_CHECK(workers < 1 || n / workers < 2147483648.0,
              "--parity reproduces riemann.cpp's int local_n: N / (P - 1) must stay below 2^31");
  double g_sum = 0.0;
  for (int w = 0; w < workers; ++w) {
    const double left = w * (range / workers);
    const double right = (w * (range / workers)) + (range / workers);
    const int local_n = static_cast<int>(n / workers);
    const double h = (right - left) / local_n;
    double sum = 0.0;
    for (int idx = 0; idx < local_n; ++idx) sum += std::sin(left + idx * h);
    g_sum += h * sum;
  }
  return g_sum;
}

double cintegrate_parity(int sp, int sm) {
  const auto& tab = profile_table();
  const int w = sp * sm;
  const int chunk = kProfileSeconds / w;
  const double dt = 1.0 / kStepsPerSec;
  // Partition arithmetic exactly as cintegrate.cu:81-97, but each thread's sum is kept in
  // long double: the reference's sequential fp64 sum of 280 000 terms carries ~1e-6 of
  // rounding noise, which lands right on the printed 6th decimal (121999.800662|6).
  long double gsum = 0.0L;
  for (int r = 0; r < w; ++r) {
    const long lo = static_cast<long>(r) * chunk * kStepsPerSec;
    const long hi = lo + static_cast<long>(chunk) * kStepsPerSec;
    long double sum = 0.0L;
    for (long i = lo; i < hi; ++i) sum += interp(tab, dt * static_cast<double>(i));
    gsum += sum / kStepsPerSec;
  }
  return static_cast<double>(gsum);
}

// 4main.c:262-269 faccel exactly as the reference evaluates it: truncating index, delta from
// the truncated time, separate multiply and add (the reference is built without FMA
// contraction; so is this, by the volatile product).
double faccel_ref(const std::vector<double>& tab, double time) {
  const int k = static_cast<int>(time);
  const double delta = time - static_cast<double>(k);
  volatile double prod = (tab[k + 1] - tab[k]) * delta;
  return tab[k] + prod;
}

TrainScanParity trainscan_parity(int P) {
  MIINT_CHECK(P >= 1, "comm size must be >= 1");
  const auto& tab = profile_table();
  const long T = static_cast<long>(kProfileSeconds) * kStepsPerSec;
  const long sub = T / P;
  const int fill_secs = kProfileSeconds / P;
  const double dt = 1.0 / kStepsPerSec;
  // Rank q's private InterpProfile is non-zero only on its fill range.
  auto interp_rank = [&](int q, long i) -> double {
    const long lo = static_cast<long>(q) * fill_secs * kStepsPerSec;
    const long hi = lo + static_cast<long>(fill_secs) * kStepsPerSec;
    return (i >= lo && i < hi) ? faccel_ref(tab, 0.0 + dt * static_cast<double>(i)) : 0.0;
  };
  // Phase 1 on root: block q = local scan of rank q's slice + carry of block q-1's last.
  std::vector<double> ds(static_cast<size_t>(T), 0.0);
  for (int q = 0; q < P; ++q) {
    double local = 0.0;
    for (long i = q * sub; i < q * sub + sub; ++i) {
      local += interp_rank(q, i);
      ds[static_cast<size_t>(i)] = local;
    }
  }
  for (int q = 1; q < P; ++q) {
    const double carry = ds[static_cast<size_t>((q - 1) * sub + sub - 1)];
    for (long i = q * sub; i < q * sub + sub; ++i) ds[static_cast<size_t>(i)] += carry;
  }
  TrainScanParity r;
  r.distance = ds[static_cast<size_t>(T - 2)] / kStepsPerSec;
  // Phase 2 (scan of the broadcast phase-1 table), root view.
  double local = 0.0, last = 0.0;
  std::vector<double> blast(P, 0.0);
  for (int q = 0; q < P; ++q) {
    local = 0.0;
    for (long i = q * sub; i < q * sub + sub; ++i) local += ds[static_cast<size_t>(i)];
    blast[q] = local;
  }
  for (int q = 0; q < P; ++q) last += blast[q];  // carries telescope to the running total
  r.sum_of_sums = last;
  return r;
}

}  // namespace oracle
}  // namespace miint
