// Host (CPU) engine: thread pool, per-ISA vector Riemann sums and the train scan on threads
// (see miint/host.hpp). The reference counterparts are the scalar loops of riemann.cpp:29-44
// and 4main.c:82-122 run by P MPI processes.
#include "miint/host.hpp"

#include <sched.h>

#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <exception>
#include <string>

#include "miint/common.hpp"
#include "miint/oracle.hpp"
#include "miint/runtime.hpp"

namespace miint {

namespace {
constexpr uint64_t kHostBlock = 4096;  // samples per compensated block (multiple of 8)

struct HostArgs {
  int integrand;
  double a, h, off;
  int ncoef;
  double coef[kMaxPolyCoeffs];
  double ts;            // TrainVel
  const double* tab;    // Table
  long nseg;
};
}  // namespace

// The same kernels three times: AVX-512 (zmm), AVX2+FMA (ymm), baseline x86-64 (xmm).
namespace hk_avx512 {
#pragma clang attribute push(__attribute__((target("avx512f,avx512dq,avx512vl,fma"))), \
                             apply_to = function)
#include "host_kernels.inc"
#pragma clang attribute pop
}  // namespace hk_avx512
namespace hk_avx2 {
#pragma clang attribute push(__attribute__((target("avx2,fma"))), apply_to = function)
#include "host_kernels.inc"
#pragma clang attribute pop
}  // namespace hk_avx2
namespace hk_base {
#include "host_kernels.inc"
}  // namespace hk_base

namespace {
enum class Isa { kAvx512, kAvx2, kBase };
Isa detect_isa() {
  // MIINT_HOST_ISA=avx2|base caps the choice (tests run every build of the kernels on one
  // AVX-512 box); it never selects an ISA the CPU lacks
  static const Isa isa = [] {
    __builtin_cpu_init();
    const char* cap = std::getenv("MIINT_HOST_ISA");
    const std::string c = cap ? cap : "";
    const bool a512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                      __builtin_cpu_supports("avx512vl");
    const bool a2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    if (a512 && c != "avx2" && c != "base") return Isa::kAvx512;
    if (a2 && c != "base") return Isa::kAvx2;
    return Isa::kBase;
  }();
  return isa;
}

double sum_slice(const HostArgs& p, uint64_t i0, uint64_t n) {
  switch (detect_isa()) {
    case Isa::kAvx512: return hk_avx512::sum_slice(p, i0, n);
    case Isa::kAvx2: return hk_avx2::sum_slice(p, i0, n);
    default: return hk_base::sum_slice(p, i0, n);
  }
}

void scan_totals(const HostArgs& p, double sps, uint64_t i0, uint64_t n, double* s1,
                 double* s2) {
  switch (detect_isa()) {
    case Isa::kAvx512: return hk_avx512::scan_totals(p, sps, i0, n, s1, s2);
    case Isa::kAvx2: return hk_avx2::scan_totals(p, sps, i0, n, s1, s2);
    default: return hk_base::scan_totals(p, sps, i0, n, s1, s2);
  }
}
}  // namespace

const char* host_isa() {
  switch (detect_isa()) {
    case Isa::kAvx512: return "avx512";
    case Isa::kAvx2: return "avx2";
    default: return "base";
  }
}

// ------------------------------------------------------------------ pool
// Default pool size: MIINT_HOST_THREADS, else OMP_NUM_THREADS (how a job's CPU share is
// usually given: the GPU pool sets it to 16 per GPU), else the CPUs this process may run
// on (sched_getaffinity), else std::thread::hardware_concurrency().
int HostPool::default_threads() {
  for (const char* k : {"MIINT_HOST_THREADS", "OMP_NUM_THREADS"}) {
    const char* v = std::getenv(k);
    if (v && std::atoi(v) > 0) return std::atoi(v);
  }
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) return CPU_COUNT(&set);
  return static_cast<int>(std::thread::hardware_concurrency());
}

HostPool::HostPool(int threads) {
  n_ = threads > 0 ? threads : default_threads();
  if (n_ < 1) n_ = 1;
  for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { worker(t); });
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

void HostPool::worker(int t) {
  long seen = 0;
  for (;;) {
    const std::function<void(int)>* job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      job = job_;
    }
    std::string err;
    try {
      (*job)(t);
    } catch (const std::exception& e) {
      err = e.what();
    } catch (...) {
      err = "unknown exception";
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (!err.empty() && err_.empty()) err_ = "host thread " + std::to_string(t) + ": " + err;
    if (--pending_ == 0) done_cv_.notify_all();
  }
}

void HostPool::run(const std::function<void(int)>& fn) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    job_ = &fn;
    pending_ = n_ - 1;
    err_.clear();
    ++gen_;
  }
  cv_.notify_all();
  std::string err;
  try {
    fn(0);
  } catch (const std::exception& e) {
    err = std::string("host thread 0: ") + e.what();
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
  job_ = nullptr;
  if (err.empty()) err = err_;
  if (!err.empty()) fail(err, __FILE__, __LINE__);
}

// ------------------------------------------------------------------ Riemann
namespace {
HostArgs make_args(const RiemannConfig& cfg, double* scale) {
  MIINT_CHECK(cfg.n >= 1, "empty rule");
  MIINT_CHECK(cfg.coef.size() <= static_cast<size_t>(kMaxPolyCoeffs), "too many coefficients");
  HostArgs p{};
  p.integrand = static_cast<int>(cfg.integrand);
  p.a = cfg.a;
  p.h = (cfg.b - cfg.a) / static_cast<double>(cfg.n);
  p.off = rule_offset(cfg.rule);
  p.ncoef = static_cast<int>(cfg.coef.size());
  for (size_t k = 0; k < cfg.coef.size(); ++k) p.coef[k] = cfg.coef[k];
  p.ts = cfg.p0;
  const std::vector<double>& tab = cfg.table.empty() ? oracle::profile_table() : cfg.table;
  MIINT_CHECK(tab.size() >= 2, "table integrand needs at least 2 entries");
  p.tab = tab.data();
  p.nseg = static_cast<long>(tab.size()) - 1;
  *scale = cfg.integrand == Integrand::kPi4 ? 4.0
           : cfg.integrand == Integrand::kTrainVel ? cfg.p1 : 1.0;
  if (cfg.integrand == Integrand::kTrainVel) MIINT_CHECK(cfg.p0 != 0.0, "train: ts must be nonzero");
  return p;
}
}  // namespace

double host_riemann(const RiemannConfig& cfg, uint64_t begin, uint64_t count, HostPool& pool) {
  MIINT_CHECK(begin + count <= cfg.n && begin + count >= begin, "host slice outside [0, n)");
  double scale = 1.0;
  const HostArgs p = make_args(cfg, &scale);
  const int T = pool.threads();
  std::vector<double> part(T, 0.0);
  pool.run([&](int t) {
    uint64_t b = 0, c = 0;
    rank_slice(count, t, T, &b, &c);
    if (c) part[t] = sum_slice(p, begin + b, c);
  });
  double s = 0.0;
  for (int t = 0; t < T; ++t) s += part[t];  // thread order
  return s * p.h * scale;
}

double host_riemann_mpi_parity(int comm_size, double n, double range, HostPool& pool) {
  const int workers = comm_size - 1;  // rank 0 only receives (P = 1 -> 0)
  if (workers < 1) return 0.0;
  // riemann.cpp:72's `int local_n = N / W` is undefined beyond INT_MAX: refused, not emulated
  MIINT_CHECK(n / workers < 2147483648.0,
              "--parity reproduces riemann.cpp's int local_n: N / (P - 1) must stay below 2^31");
  std::vector<double> part(workers, 0.0);
  const int T = pool.threads();
  pool.run([&](int t) {
    for (int w = t; w < workers; w += T) {  // the loop of riemann.cpp:29-44, as written
      const double left = w * (range / workers);
      const double right = (w * (range / workers)) + (range / workers);
      const int local_n = static_cast<int>(n / workers);
      const double h = (right - left) / local_n;
      double sum = 0.0;
      for (int idx = 0; idx < local_n; ++idx) sum += std::sin(left + idx * h);
      part[w] = h * sum;
    }
  });
  double g_sum = 0.0;
  for (int w = 0; w < workers; ++w) g_sum += part[w];  // MPI_Recv in rank order
  return g_sum;
}

// ------------------------------------------------------------------ train scan
HostScanResult host_trainscan(const HostScanConfig& cfg, HostPool& pool, HostComm* comm,
                              std::vector<double>* vel, std::vector<double>* pos) {
  MIINT_CHECK(cfg.steps_per_sec >= 1 && cfg.seconds >= 1, "bad train-scan size");
  const double w0 = wall_seconds();
  const int rank = comm ? comm->rank() : 0, world = comm ? comm->world() : 1;
  const uint64_t total = static_cast<uint64_t>(cfg.steps_per_sec) * cfg.seconds;
  HostScanResult r;
  rank_slice(total, rank, world, &r.begin, &r.count);
  MIINT_CHECK(r.count >= 1, "empty train-scan slice");
  const std::vector<double>& tab = cfg.table.empty() ? oracle::profile_table() : cfg.table;
  MIINT_CHECK(tab.size() >= 2 && static_cast<size_t>(cfg.seconds) <= tab.size() - 1,
              "train scan: seconds exceeds the table");
  HostArgs p{};
  p.integrand = static_cast<int>(Integrand::kTable);
  p.tab = tab.data();
  p.nseg = static_cast<long>(tab.size()) - 1;
  const double sps = cfg.steps_per_sec, dt = 1.0 / sps;
  const int T = pool.threads();
  std::vector<double> s1(T, 0.0), s2(T, 0.0), cnt(T, 0.0);
  // pass 1: per-thread {sum v, sum of the thread's running sums}
  pool.run([&](int t) {
    uint64_t b = 0, c = 0;
    rank_slice(r.count, t, T, &b, &c);
    cnt[t] = static_cast<double>(c);
    if (c) scan_totals(p, sps, r.begin + b, c, &s1[t], &s2[t]);
  });
  // segments compose as (V, P) + (S1, S2, n) = (V + S1, P + S2 + n V)
  double rv = 0.0, rp = 0.0, rn = 0.0;  // this rank's totals
  for (int t = 0; t < T; ++t) {
    rp += s2[t] + cnt[t] * rv;
    rv += s1[t];
    rn += cnt[t];
  }
  double cv = 0.0, cp = 0.0, gv = rv, gp = rp;  // carries into this rank; global totals
  if (world > 1) {
    std::vector<double> all(3 * static_cast<size_t>(world));
    const double mine[3] = {rv, rp, rn};
    comm->allgather(mine, all.data(), 3);
    gv = gp = 0.0;
    for (int q = 0; q < world; ++q) {
      if (q == rank) {
        cv = gv;
        cp = gp;
      }
      gp += all[3 * q + 1] + all[3 * q + 2] * gv;
      gv += all[3 * q];
    }
  }
  // pass 2: the running integral and its running integral with every carry applied
  if (cfg.keep || vel || pos) {
    std::vector<double> own_v, own_p;
    std::vector<double>& V = vel ? *vel : own_v;
    std::vector<double>& P = pos ? *pos : own_p;
    V.assign(r.count, 0.0);
    P.assign(r.count, 0.0);
    std::vector<double> tv(T), tp(T);  // per-thread carries
    double av = cv, ap = cp;
    for (int t = 0; t < T; ++t) {
      tv[t] = av;
      tp[t] = ap;
      ap += s2[t] + cnt[t] * av;
      av += s1[t];
    }
    pool.run([&](int t) {
      uint64_t b = 0, c = 0;
      rank_slice(r.count, t, T, &b, &c);
      // compensated running sums (a plain 18e6-term running sum drifts by ~1e-10 relative,
      // which is how the reference's printed values drift: 122000.004030)
      double v1 = tv[t], v2 = tp[t], c1 = 0.0, c2 = 0.0;
      const double* tb = tab.data();
      const long nseg = p.nseg;
      for (uint64_t k = 0; k < c; ++k) {  // the sample of host_kernels.inc train_sample
        const double idx = static_cast<double>(r.begin + b + k);
        const double sg = std::min(std::floor((idx + 0.5) * (1.0 / sps)),
                                   static_cast<double>(nseg - 1));
        const long i = static_cast<long>(sg);
        const double v = std::fma(tb[i + 1] - tb[i], (idx - sg * sps) * dt, tb[i]);
        double y = v - c1, u = v1 + y;
        c1 = (u - v1) - y;
        v1 = u;
        y = v1 - c2;
        u = v2 + y;
        c2 = (u - v2) - y;
        v2 = u;
        V[b + k] = v1;
        P[b + k] = v2;
      }
    });
  }
  r.distance = gv / cfg.steps_per_sec;
  r.sum_of_sums = gp;
  r.seconds = wall_seconds() - w0;
  return r;
}

}  // namespace miint
