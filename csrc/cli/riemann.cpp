// riemann — Riemann sum of sin(x) on [0, pi] (reference: riemann.cpp, MPI master/worker).
//
// Default output is the reference's two lines (riemann.cpp:92-96):
//   %lf seconds
//   The integral of f(x) from 0.0 to <b> with <n> steps is <sum>      (precision 15)
// Differences by design: every GPU works (the reference's rank 0 only receives, so P
// processes give P-1 workers and P=1 prints 0 — SURVEY B10); the partial sums meet in one
// RCCL all-reduce instead of P-1 MPI_Send/Recv pairs; N is 64-bit (1e10 works, B9).
// --parity runs the master/worker program itself on the GPUs: under P ranks (miintrun -np P,
// torchrun, --gpus P, --loopback P) rank 0 coordinates and integrates nothing, rank r >= 1
// integrates worker r-1's (int)(N/W) samples on its own GPU, the partials meet in one
// allgather and rank 0 adds them in rank order (P=1 -> 0).
//
// Timing: every rank's clock starts after a collective barrier and the reported time is the
// slowest rank's (max over the communicator); --json (or --one-shot) also measures and reports
// ms_one_shot, one integration per call from launch to the result in pinned host memory
// (median). The default program does not: it is the reference's one run.
//
// --device cpu runs the reference's own side of the comparison natively on the host: every
// rank (process) integrates its slice on --threads T vector threads (miint/host.hpp), and
// the ranks' partials meet in a rank-order host all-reduce; --parity emulates --ranks P
// master/worker ranks (riemann.cpp:65-86) in this process.
//
// --expr "EXPR" integrates any f(x) given as one C++ expression over x (HIP device math:
// sin, exp, pow, ...), compiled at run time for gfx950 with hipRTC (miint/expr.hpp) — where
// the reference edits riemann.cpp:37 and recompiles; with --device cpu, compiled for the
// host cores instead (HostExpr). --analytic V adds the error vs V.
//
//   ./riemann [--n 1e9] [--gpus G] [--integrand sin|pi4|poly|train] [--rule left|mid|right]
//             [--dtype fp64|fp32|fp32acc] [--iters K] [--block 64..1024] [--grid G] [--parity]
//             [--json] [--jsonl FILE]
//             [--device cpu [--threads T] [--ranks P]] [--expr EXPR --a A --b B [--analytic V]]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <memory>
#include <sstream>
#include <vector>

#include "cli_common.hpp"
#include "miint/expr.hpp"
#include "miint/fault.hpp"
#include "miint/host.hpp"
#include "miint/integrator.hpp"
#include "miint/oracle.hpp"
#include "miint/trace.hpp"

using namespace miint;

namespace {

void print_result(double secs, double hi, double nd, double result) {
  std::printf("%lf seconds\n", secs);
  std::cout.precision(15);
  std::cout << "The integral of f(x) from 0.0 to " << hi << " with " << nd << " steps is "
            << result << std::endl;
}

// --device cpu (see the header comment).
int run_host(const cli::Args& a, const RiemannConfig& cfg, double nd, int iters) {
  cli::HostRanks hr = cli::host_ranks(a);
  HostPool pool(hr.threads);
  double result = 0.0, host_ms = 0.0;
  int ranks = hr.world;
  if (a.flag("parity")) {
    // riemann.cpp:65-86 as the reference runs it: P ranks -> P-1 workers on host threads,
    // scalar libm sin and sequential sums, rank-order gather; P = 1 -> 0 (B10)
    MIINT_CHECK(hr.world == 1, "--device cpu --parity emulates --ranks P in one process");
    MIINT_CHECK(cfg.integrand == Integrand::kSin && cfg.a == 0.0,
                "--device cpu --parity is the reference's sin on [0, b] program");
    ranks = static_cast<int>(a.integer("ranks", 8));
    MIINT_CHECK(ranks >= 1, "--ranks must be >= 1");
    const double t0 = wall_seconds();
    result = host_riemann_mpi_parity(ranks, nd, cfg.b, pool);
    host_ms = (wall_seconds() - t0) * 1e3;
  } else {
    uint64_t b = 0, c = 0;
    rank_slice(cfg.n, hr.rank, hr.world, &b, &c);
    for (int i = 0; i < iters; ++i) {  // best of --iters
      if (hr.comm) hr.comm->barrier();
      const double t0 = wall_seconds();
      double v = c ? host_riemann(cfg, b, c, pool) : 0.0;
      if (hr.comm) hr.comm->allreduce_sum(&v, 1);
      fault::delay(hr.rank);  // MIINT_FAULT_*: a slow rank (agreement tests)
      const double ms = (wall_seconds() - t0) * 1e3;
      if (i == 0 || ms < host_ms) host_ms = ms;
      result = v;
    }
    if (hr.comm) {  // the slowest rank's time
      double t = -host_ms;
      std::vector<double> all(hr.world);
      hr.comm->allgather(&t, all.data(), 1);
      for (double x : all) host_ms = std::max(host_ms, -x);
    }
  }
  if (hr.rank != 0) return 0;
  const double secs = wall_seconds() - process_start_seconds();
  print_result(secs, cfg.b, nd, result);
  const double exact = cfg.integrand == Integrand::kTable
                           ? oracle::table_integral(cfg.table, cfg.a, cfg.b)
                           : oracle::analytic(cfg.integrand, cfg.a, cfg.b, cfg.coef, cfg.p0, cfg.p1);
  cli::emit(a, cli::JsonRecord()
                   .add("program", "riemann")
                   .add("device", "cpu")
                   .add("isa", host_isa())
                   .add("integrand", a.str("integrand", "sin"))
                   .add("dtype", "fp64")
                   .add("rule", a.str("rule", "left"))
                   .add("n", nd)
                   .add("ranks", ranks)
                   .add("threads_per_rank", pool.threads())
                   .add("parity", a.flag("parity"))
                   .add("result", result)
                   .add("analytic", exact)
                   .add("abs_err", std::fabs(result - exact))
                   .add("rel_err", std::fabs(result - exact) / std::fabs(exact))
                   .add("host_ms", host_ms)
                   .add("subintervals_per_s", host_ms > 0 ? nd / (host_ms * 1e-3) : 0.0)
                   .add("seconds_wall", secs));
  return 0;
}

// --expr --device cpu: host ranks, f compiled for the host cores (HostExpr).
int run_host_expr(const cli::Args& a, const RiemannConfig& cfg, double nd, int iters) {
  const std::string expr = a.str("expr", "");
  cli::HostRanks hr = cli::host_ranks(a);
  HostPool pool(hr.threads);
  const HostExpr he(expr);
  uint64_t b = 0, c = 0;
  rank_slice(cfg.n, hr.rank, hr.world, &b, &c);
  double result = 0.0, host_ms = 0.0;
  for (int i = 0; i < iters; ++i) {  // best of --iters
    if (hr.comm) hr.comm->barrier();
    const double t0 = wall_seconds();
    double v = c ? he.integrate(cfg.a, cfg.b, cfg.n, cfg.rule, b, c, pool) : 0.0;
    if (hr.comm) hr.comm->allreduce_sum(&v, 1);
    const double ms = (wall_seconds() - t0) * 1e3;
    if (i == 0 || ms < host_ms) host_ms = ms;
    result = v;
  }
  if (hr.rank != 0) return 0;
  const double secs = wall_seconds() - process_start_seconds();
  print_result(secs, cfg.b, nd, result);
  cli::JsonRecord r;
  r.add("program", "riemann").add("device", "cpu").add("expr", expr).add("a", cfg.a)
      .add("b", cfg.b).add("n", nd).add("rule", a.str("rule", "left")).add("ranks", hr.world)
      .add("threads_per_rank", pool.threads()).add("result", result);
  if (a.has("analytic")) {
    const double exact = a.num("analytic", 0.0);
    r.add("analytic", exact).add("abs_err", std::fabs(result - exact));
  }
  cli::emit(a, r.add("host_ms", host_ms)
                   .add("subintervals_per_s", host_ms > 0 ? nd / (host_ms * 1e-3) : 0.0)
                   .add("seconds_wall", secs));
  return 0;
}

// --expr (see the header comment): GPU ranks as in the default path, f compiled by hipRTC.
int run_expr(const cli::Args& a, const RiemannConfig& cfg, double nd, int iters) {
  if (cli::on_cpu(a)) return run_host_expr(a, cfg, nd, iters);
  const std::string expr = a.str("expr", "");
  const cli::Topology topo = cli::topology(a);
  double result = 0.0, dev_ms = 0.0;
  std::mutex mu;
  cli::RankFacts facts;
  cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
    ExprIntegrator ei(expr, dev);
    RankAgree agree(comm);
    uint64_t b = 0, c = 0;
    rank_slice(cfg.n, rank, topo.world, &b, &c);
    const double v = ei.integrate(cfg.a, cfg.b, cfg.n, cfg.rule, b, c, 1.0, comm);
    // barrier right before the clock starts; the slowest rank's time
    const double ms = agree.max(ei.time(cfg.a, cfg.b, cfg.n, cfg.rule, b, c, iters,
                                        [&] { agree.barrier(); }, [&] { fault::delay(rank); }));
    std::lock_guard<std::mutex> g(mu);
    if (rank == topo.rank0) {
      result = v;
      dev_ms = ms;
      facts.note(comm);
    }
  });
  if (topo.rank0 != 0) return 0;
  const double secs = wall_seconds() - process_start_seconds();
  print_result(secs, cfg.b, nd, result);
  cli::JsonRecord r;
  r.add("program", "riemann")
      .add("expr", expr)
      .add("a", cfg.a)
      .add("b", cfg.b)
      .add("n", nd)
      .add("rule", a.str("rule", "left"))
      .add("gpus", topo.world)
      .add("result", result);
  facts.add(r, topo);
  if (a.has("analytic")) {
    const double exact = a.num("analytic", 0.0);
    r.add("analytic", exact).add("abs_err", std::fabs(result - exact));
  }
  cli::emit(a, r.add("device_ms", dev_ms)
                   .add("subintervals_per_s", dev_ms > 0 ? nd / (dev_ms * 1e-3) : 0.0)
                   .add("seconds_wall", secs));
  return 0;
}

}  // namespace

constexpr const char* kUsage =
    "usage: riemann [--n 1e9] [--gpus G] [--loopback W] [--integrand sin|pi4|poly|train|table]\n"
    "               [--rule left|mid|right] [--dtype fp64|fp32|fp32acc] [--div series_exact|series|ieee]\n"
    "               [--iters K] [--block 64..1024] [--grid G] [--a A --b B] [--parity]\n"
    "               [--one-shot | --no-one-shot] [--no-multistep] [--unfused]\n"
    "               [--json] [--jsonl FILE] [--profile FILE]\n"
    "               [--device cpu [--threads T] [--ranks P]]\n"
    "               [--expr EXPR --a A --b B [--analytic V]]\n"
    "Riemann sum of f on [a, b] (default sin on [0, pi], N = 1e9); prints the reference's\n"
    "two lines, or one JSON record with --json. Multi-GPU: --gpus G, torchrun or miintrun.\n";

int main(int argc, char** argv) {
  try {
    install_crash_handler_from_env();
    cli::Args a(argc, argv);
    if (cli::usage_requested(a, kUsage)) return 0;
    const Integrand f = cli::parse_integrand(a.str("integrand", "sin"));
    const double pi = 3.14159265358979323846;
    double lo = 0.0, hi = pi;  // riemann.cpp:6 RANGE = M_PI
    if (f == Integrand::kPi4) hi = 1.0;
    std::vector<double> prof;  // table integrand: --profile FILE or the built-in profile
    if (f == Integrand::kTable)
      prof = a.has("profile") ? oracle::load_profile(a.str("profile", "")) : oracle::profile_table();
    if (f == Integrand::kTrainVel) hi = 1800.0;
    if (f == Integrand::kTable) hi = static_cast<double>(prof.size() - 1);
    lo = a.num("a", lo);
    hi = a.num("b", hi);
    const double nd = a.num("n", 1e9);  // riemann.cpp:10 STEPS
    const auto n = static_cast<uint64_t>(nd);
    const int iters = static_cast<int>(a.integer("iters", 1));
    MIINT_CHECK(iters >= 1, "--iters must be >= 1");

    RiemannConfig cfg;
    cfg.integrand = f;
    cfg.a = lo;
    cfg.b = hi;
    cfg.n = n;
    cfg.rule = cli::parse_rule(a.str("rule", "left"));
    cfg.dtype = cli::parse_dtype(a.str("dtype", "fp64"));
    cfg.div = cli::parse_div(a.str("div", "series_exact"));
    cfg.fused = !a.flag("unfused");
    cfg.multistep = !a.flag("no-multistep");  // chained batches, full auto grid
    // --block: threads per workgroup (the reference's SP, cintegrate.cu:17-18); --grid:
    // workgroups (its SM), 0 = auto
    cfg.block = static_cast<int>(a.integer("block", kRiemannBlock));
    cfg.grid = static_cast<int>(a.integer("grid", 0));
    MIINT_CHECK(riemann_block_ok(cfg.block), "--block must be 64, 128, 256, 512 or 1024");
    if (f == Integrand::kTrainVel) { cfg.p0 = oracle::kTrainTs; cfg.p1 = oracle::kTrainVs; }
    if (f == Integrand::kTable) cfg.table = prof;
    if (f == Integrand::kPoly) cfg.coef = {1.0, -0.5, 0.25, 0.125};

    if (a.has("expr")) return run_expr(a, cfg, nd, iters);
    if (cli::on_cpu(a)) return run_host(a, cfg, nd, iters);
    const cli::Topology topo = cli::topology(a);

    double result = 0.0, dev_ms = 0.0, wall_ms = 0.0, one_shot_ms = 0.0;
    // The one-integration-per-call harness (~450 extra integrations) runs only for a record
    // (--json) or when asked (--one-shot): the default program is the reference's single run,
    // one cold + one timed integration before its "seconds" line (riemann.cpp:49-51,90-96)
    const bool one_shot = (a.flag("json") || a.flag("one-shot")) && !a.flag("no-one-shot");
    LaunchShape launch_shape{0, cfg.block};
    cli::RankFacts facts;
    std::mutex mu;
    std::vector<double> partials;  // --parity: the workers' partials, rank order
    if (a.flag("parity")) {
      // riemann.cpp:62-86 as a distributed program: P = world ranks -> W = P - 1 workers. Rank
      // 0 is the coordinator and integrates nothing; rank r >= 1 integrates worker r-1's
      // slice [(r-1) R/W, r R/W) with (int)(N / W) samples on its own GPU; the partials meet
      // in one allgather and rank 0 adds them in rank order (the MPI_Recv loop's rounding,
      // riemann.cpp:82-85). P = 1: no workers, the sum is 0 (B10).
      const int P = topo.world;
      const int W = P - 1;
      MIINT_CHECK(W < 1 || nd / W < 2147483648.0,
                  "--parity reproduces riemann.cpp's int local_n: N / (P - 1) must stay below 2^31");
      cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
        RankAgree agree(comm);
        std::unique_ptr<RiemannPlan> plan;
        if (rank >= 1) {
          RiemannConfig c = cfg;
          const int w = rank - 1;
          c.a = w * ((hi - lo) / W);
          c.b = c.a + (hi - lo) / W;
          c.n = static_cast<uint64_t>(static_cast<int>(nd / W));
          c.multistep = false;  // one integration: the full grid, one fused launch
          plan.reset(new RiemannPlan(c, dev));  // the worker's own; the partials meet below
          plan->run();                          // cold: code-object load, first launch
        }
        double partial = 0.0;
        std::vector<double> best;
        for (int it = 0; it < iters; ++it) {
          agree.barrier();
          const double t0 = wall_seconds();
          if (plan) partial = plan->run();
          const std::vector<double> all = agree.gather({partial});  // MPI_Send / MPI_Recv
          fault::delay(rank);
          best.push_back(agree.max((wall_seconds() - t0) * 1e3));
          if (rank == topo.rank0 && it + 1 == iters) {
            double g_sum = 0.0;
            for (int q = 1; q < P; ++q) g_sum += all[static_cast<size_t>(q)];  // rank order
            std::lock_guard<std::mutex> g(mu);
            result = g_sum;
            partials.assign(all.begin(), all.end());
          }
        }
        std::lock_guard<std::mutex> g(mu);
        if (rank == topo.rank0) {
          dev_ms = *std::min_element(best.begin(), best.end());
          wall_ms = dev_ms;
          facts.note(comm);
          if (plan) launch_shape = plan->shape();
        }
      });
    } else {
      cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
        RiemannPlan plan(cfg, dev, comm);
        RankAgree agree(comm);
        if (a.has("prepare")) plan.prepare_steps(static_cast<int>(a.integer("prepare", iters)));
        plan.run_steps(1, comm != nullptr, false);  // cold: code-object load, first launch
        // the timed steps: every rank's clock starts after a collective barrier, the time
        // reported is the slowest rank's (the reference's rank 0 stops its clock only after
        // every worker's result has arrived, riemann.cpp:82-93)
        StepTiming t = plan.run_steps(iters, comm != nullptr, iters > 1);
        const double ms = agree.max(t.device_ms / iters);
        const double wms = agree.max(t.wall_s * 1e3 / iters);
        const double v = plan.host_result(plan.host_index_of(iters - 1, iters > 1));
        // one integration per call, launch to pinned result (the reference's own timing unit)
        double shot = 0.0;
        if (one_shot) {
          if (!plan.collective()) {
            // 400 settling calls first: from idle the clocks take ~250 calls to settle. A
            // 1-step graph replay with the host polling the pinned result: the fastest form
            // (profiles/r4/one_shot_grid_settled.jsonl: 78.4-79 us against 80.1 direct_poll)
            try {
              shot = plan.time_one_shot(50, plan.direct() ? "graph_poll" : "direct", 400)
                         .median_us * 1e-3;
            } catch (const Error&) {
              // only a failed 1-step graph capture falls back to the direct launch; any other
              // failure (a replay whose value disagrees, a result never stored) propagates
              if (!plan.direct() || plan.graph_error().empty()) throw;
              shot = plan.time_one_shot(50, "direct_poll", 400).median_us * 1e-3;
            }
          } else {
            std::vector<double> v1;
            for (int k = 0; k < 10; ++k) v1.push_back(plan.run_steps(1, true, false).wall_s * 1e3);
            shot = agree.max(cli::median(v1));
          }
        }
        std::lock_guard<std::mutex> g(mu);
        if (rank == topo.rank0) {
          launch_shape = plan.shape();
          result = v;
          dev_ms = ms;
          wall_ms = wms;
          one_shot_ms = shot;
          facts.note(comm);
        }
      });
    }
    if (topo.rank0 != 0) return 0;
    const double secs = wall_seconds() - process_start_seconds();
    print_result(secs, hi, nd, result);
    const double exact = f == Integrand::kTable ? oracle::table_integral(prof, lo, hi)
                                                : oracle::analytic(f, lo, hi, cfg.coef, cfg.p0, cfg.p1);
    cli::JsonRecord rec;
    rec.add("program", "riemann")
        .add("integrand", a.str("integrand", "sin"))
        .add("dtype", a.str("dtype", "fp64"))
        .add("rule", a.str("rule", "left"))
        .add("n", nd)
        .add("gpus", topo.world)
        .add("parity", a.flag("parity"));
    facts.add(rec, topo);
    // --parity integrates W (int)(N / W) samples (fewer than N when W does not divide N)
    const int workers = topo.world - 1;
    const double work =
        !a.flag("parity") ? nd
                          : (workers >= 1 ? static_cast<double>(workers) *
                                                static_cast<int>(nd / workers)
                                          : 0.0);
    if (a.flag("parity")) {
      // the partials in rank order (rank 0, the coordinator, contributes 0)
      std::string ps = "[";
      for (size_t q = 0; q < partials.size(); ++q) {
        char b[40];
        std::snprintf(b, sizeof b, "%s%.17g", q ? "," : "", partials[q]);
        ps += b;
      }
      rec.add("workers", workers).add("samples", work).add_raw("partials", ps + "]");
    }
    rec.add("result", result)
        .add("analytic", exact)
        .add("abs_err", std::fabs(result - exact))
        .add("rel_err", std::fabs(result - exact) / std::fabs(exact))
        .add("block", launch_shape.block)
        .add("grid", launch_shape.grid)
        .add("device_ms", dev_ms)
        .add("seconds_device", dev_ms * 1e-3)
        .add("wall_ms_per_integration", wall_ms)
        .add("timing", a.flag("parity") ? "host, barrier to gathered partials, slowest rank"
                                        : "hipEvent per integration, slowest rank")
        .add("subintervals_per_s", dev_ms > 0 ? work / (dev_ms * 1e-3) : 0.0);
    rec.add("one_shot", one_shot && !a.flag("parity"));
    if (!a.flag("parity") && one_shot) rec.add("ms_one_shot", one_shot_ms);
    cli::emit(a, rec.add("seconds_wall", secs));
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "riemann: %s\n", e.what());
    return 1;
  }
}
