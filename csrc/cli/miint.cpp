// miint — unified native driver: device info, benchmark sweeps, oracle self-checks.
//
//   ./miint info
//   ./miint bench [--integrand pi4] [--n 1e9] [--dtype fp64] [--rule left] [--iters 200]
//                 [--gpus G] [--div series_exact|series|ieee] [--unfused] [--no-graph]      (JSON lines)
//   ./miint sweep [--gpus G]     N in {1e6,1e9,1e10} x dtype {fp64,fp32} x integrand
//   ./miint table2d [--grid 4096] [--gpus G] [--slice R/W] [--no-graph]
//                                2-D velocity-field integral (BASELINE #5); timed as
//                                replays of a hipGraph of 32 integrations
//   ./miint selfcheck            every SURVEY §6.1 oracle on the GPU, exit 1 on mismatch
//   ./miint comm [--gpus G] [--max-bytes 144e6] [--iters 20]
//                                RCCL allreduce / allgather / broadcast sweep, 8 B .. 144 MB
// Every record is one JSON line on stdout; --jsonl FILE also appends it to FILE.
//
// The reference has no benchmark harness (its only artefact is a wall-clock
// "%lf seconds" line covering process start to print); this tool reports device time per
// integration from hipEvents around graph replays, plus subintervals/s and |error|.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "cli_common.hpp"
#include "miint/integrator.hpp"
#include "miint/oracle.hpp"
#include "miint/table2d.hpp"
#include "miint/trainscan.hpp"

using namespace miint;

namespace {

struct BenchRow {
  std::string integrand, dtype, rule;
  double n = 0, result = 0, exact = 0, ms = 0;
  int gpus = 1;
  int block = 0, grid = 0;  // launch shape of rank 0's plan
  bool multistep = false, close_in_launch = false, allreduce_to_host = false;
  BatchDiag diag;  // --diagnose: rank 0's diagnostic batch (diag.steps == 0 otherwise)
  cli::RankFacts facts;
  cli::Topology topo;
};

Integrand integrand_of(const std::string& s) { return cli::parse_integrand(s); }

RiemannConfig make_cfg(const std::string& integ, double n, const std::string& dtype,
                       const std::string& rule, const std::string& div) {
  RiemannConfig c;
  c.integrand = integrand_of(integ);
  c.a = 0.0;
  c.b = c.integrand == Integrand::kPi4 || c.integrand == Integrand::kPoly ? 1.0
      : c.integrand == Integrand::kSin ? 3.14159265358979323846 : 1800.0;
  c.n = static_cast<uint64_t>(n);
  c.dtype = cli::parse_dtype(dtype);
  c.rule = cli::parse_rule(rule);
  c.div = cli::parse_div(div);
  if (c.integrand == Integrand::kTrainVel) { c.p0 = oracle::kTrainTs; c.p1 = oracle::kTrainVs; }
  if (c.integrand == Integrand::kTable) c.table = oracle::profile_table();
  if (c.integrand == Integrand::kPoly) c.coef = {0.3, -1.2, 0.7, 0.05, -0.4, 0.9, 0.1};
  return c;
}

BenchRow bench_one(const cli::Topology& topo, RiemannConfig cfg, int iters, bool graphs,
                   int settle_steps = -1, bool diagnose = false) {
  BenchRow row;
  row.n = static_cast<double>(cfg.n);
  row.gpus = topo.world;
  row.exact = oracle::analytic(cfg.integrand, cfg.a, cfg.b, cfg.coef, cfg.p0, cfg.p1);
  row.topo = topo;
  std::mutex mu;
  cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
    RiemannPlan plan(cfg, dev, comm);
    RankAgree agree(comm);
    plan.run_steps(3, comm != nullptr, graphs);  // warmup + capture
    // Clock settle (see bench.py): ~60 ms of back-to-back steps before timing. The count is
    // a function of the rank's sample count only, so every rank issues the same collectives.
    const double est_s = static_cast<double>(plan.count()) / 1.3e13;
    const int settle = settle_steps >= 0 ? settle_steps
                       : static_cast<int>(std::min(20000.0, std::max(3.0, 0.06 / est_s)));
    plan.run_steps(settle, comm != nullptr, graphs);
    // barrier before every rank's clock (run_steps), the slowest rank's time over all ranks
    // of the communicator (not only this process's)
    StepTiming t = plan.run_steps(iters, comm != nullptr, graphs);
    const double ms = agree.max(t.wall_s * 1e3 / iters);
    // untimed, after the clock: one batch of min(iters, slots) steps split into its stages
    // (RiemannPlan::diagnose_batch; every rank runs it, it has barriers of its own)
    BatchDiag d;
    if (diagnose) d = plan.diagnose_batch(std::min(iters, plan.config().slots));
    std::lock_guard<std::mutex> g(mu);
    if (ms > row.ms) row.ms = ms;
    if (rank == topo.rank0) {
      row.facts.note(comm);
      row.result = plan.host_result(plan.host_index_of(iters - 1, graphs));
      row.block = plan.shape().block;
      row.grid = plan.shape().grid;
      row.multistep = plan.multistep();
      row.close_in_launch = plan.close_in_launch();
      row.allreduce_to_host = plan.allreduce_to_host();
      row.diag = d;
    }
  });
  return row;
}

void print_row(const cli::Args& a, const BenchRow& r, const char* integ, const char* dtype,
               const char* rule) {
  cli::JsonRecord rec;
  rec.add("integrand", integ).add("dtype", dtype).add("rule", rule).add("n", r.n).add("gpus", r.gpus);
  r.facts.add(rec, r.topo);
  rec.add("block", r.block)
                   .add("grid", r.grid)
                   .add("multistep", r.multistep)
                   .add("close_in_launch", r.close_in_launch)
                   .add("allreduce_to_host", r.allreduce_to_host)
                   .add("ms_per_integration", r.ms)
                   .add("subintervals_per_s", r.n / (r.ms * 1e-3))
                   .add("result", r.result)
                   .add("analytic", r.exact)
                   .add("abs_err", std::fabs(r.result - r.exact));
  if (r.diag.steps > 0)
    rec.add("diag_steps", r.diag.steps)
        .add("diag_compute_us", r.diag.compute_us)
        .add("diag_close_us", r.diag.close_us)
        .add("diag_allreduce_us", r.diag.allreduce_us)
        .add("diag_copy_us", r.diag.copy_us)
        .add("diag_tail_us", r.diag.tail_us())
        .add("diag_boundary_us", r.diag.boundary_us())
        .add("diag_device_us", r.diag.device_us)
        .add("diag_marker_us", r.diag.marker_us)
        .add("diag_host_us", r.diag.wall_us - r.diag.device_us);
  cli::emit(a, rec, true);
}

int selfcheck() {
  int bad = 0;
  auto check = [&](const char* what, double got, double want, double tol) {
    const bool ok = std::fabs(got - want) <= tol;
    std::printf("%-44s got %.9f want %.9f  %s\n", what, got, want, ok ? "ok" : "MISMATCH");
    bad += !ok;
  };
  {
    RiemannPlan p(make_cfg("pi4", 1e9, "fp64", "left", "series"), 0);
    check("pi4 left N=1e9 (|err| = h)", p.run(), 3.14159265358979323846 + 1e-9, 2e-12);
  }
  {
    RiemannPlan p(make_cfg("pi4", 1e9, "fp64", "mid", "series"), 0);
    check("pi4 mid N=1e9", p.run(), 3.14159265358979323846, 1e-13);
  }
  {
    RiemannPlan p(make_cfg("sin", 1e9, "fp64", "left", "series"), 0);
    check("sin [0,pi] N=1e9", p.run(), 2.0, 1e-12);
  }
  {
    RiemannConfig c = make_cfg("table", 18e6, "fp64", "left", "series");
    RiemannPlan p(c, 0);
    // exact for the piecewise-linear profile sampled on its own knots: 122000.004000
    // (the reference prints ...004030: sequential-fp64 rounding over 18e6 running sums)
    check("cintegrate full coverage", p.run(), 122000.004000, 1e-6);
    c.b = 1792.0;
    c.n = 17920000;
    RiemannPlan q(c, 0);
    check("cintegrate --parity (SP=32,SM=2)", q.run(), 121999.800663, 5e-6);
  }
  {
    TrainScanConfig tc;
    TrainScan ts(tc, 0);
    const TrainScanResult r = ts.run();
    check("trainscan distance (P=1)", r.distance, 122000.004000, 1e-6);
  }
  std::printf("%s\n", bad ? "SELFCHECK FAILED" : "SELFCHECK OK");
  return bad ? 1 : 0;
}

// RCCL collective sweep (SURVEY §7.1 layer 7): the payloads the framework actually moves
// (8 B Riemann partials, P x 8 B scan carries, the 144 MB table of 4main.c:157) and the sizes
// between them. Algorithm bandwidth = bytes a rank ends up with / time; bus bandwidth uses
// the usual ring factors (allreduce 2(P-1)/P, allgather (P-1)/P, broadcast 1), so it is the
// per-link rate to compare against one xGMI link. Times are the slowest rank's.
int comm_sweep(const cli::Args& a, const cli::Topology& topo, double max_bytes, int iters) {
  std::vector<size_t> counts;  // doubles per rank
  for (size_t c = 1; c * 8.0 <= max_bytes; c *= 8) counts.push_back(c);
  if (counts.empty() || counts.back() * 8.0 < max_bytes) counts.push_back(static_cast<size_t>(max_bytes / 8));
  const char* ops[] = {"allreduce", "allgather", "broadcast"};
  std::vector<double> ms(counts.size() * 3, 0.0);
  std::mutex mu;
  auto body = [&](int /*rank*/, int dev, const Comm* comm) {
    DeviceGuard g(dev);
    Stream s;
    RankAgree agree(comm);  // each op's time is the slowest rank's, over every process
    const size_t cmax = counts.back();
    DeviceBuffer<double> a(cmax), b(cmax * static_cast<size_t>(comm->world()));
    MIINT_HIP(hipMemsetAsync(a.get(), 0, a.bytes(), s.get()));
    Event e0, e1;
    for (size_t k = 0; k < counts.size(); ++k)
      for (int op = 0; op < 3; ++op) {
        auto issue = [&] {
          if (op == 0) comm->allreduce_sum(a.get(), b.get(), counts[k], s.get());
          else if (op == 1) comm->allgather(a.get(), b.get(), counts[k], s.get());
          else comm->broadcast(a.get(), counts[k], 0, s.get());
        };
        for (int w = 0; w < 3; ++w) issue();
        s.sync();
        agree.barrier();
        e0.record(s.get());
        for (int i = 0; i < iters; ++i) issue();
        e1.record(s.get());
        e1.sync();
        comm->check_async();
        const double t = agree.max(Event::elapsed_ms(e0, e1) / iters);
        std::lock_guard<std::mutex> l(mu);
        ms[k * 3 + op] = std::max(ms[k * 3 + op], t);
      }
  };
  capture_rccl_log();
  if (!topo.multiproc && topo.world == 1) {
    auto one = RcclComm::init_all({0});
    body(0, 0, one[0].get());
  } else {
    cli::run_ranks(topo, body);
  }
  if (topo.rank0 != 0) return 0;
  const double P = topo.world;
  const RcclTransport tr = rccl_transport();  // the connections the sweep's collectives used
  const bool share = ranks_share_devices() && topo.world > 1;
  const std::string terr = transport_error(
      tr, topo.world, topo.multiproc ? cli::env_int("LOCAL_WORLD_SIZE", topo.world) : topo.world,
      share);
  if (!terr.empty()) std::fprintf(stderr, "miint comm: transport check: %s\n", terr.c_str());
  for (size_t k = 0; k < counts.size(); ++k)
    for (int op = 0; op < 3; ++op) {
      const double bytes = counts[k] * 8.0 * (op == 1 ? P : 1.0);
      const double t = ms[k * 3 + op];
      const double alg = bytes / (t * 1e-3) / 1e9;
      const double factor = op == 0 ? 2.0 * (P - 1) / P : (op == 1 ? (P - 1) / P : 1.0);
      cli::emit(a, cli::JsonRecord()
                       .add("op", ops[op])
                       .add("gpus", topo.world)
                       .add("bytes", bytes)
                       .add("us", t * 1e3)
                       .add("algbw_GBps", alg)
                       .add("busbw_GBps", alg * factor)
                       .add("ranks_share_gpus", ranks_share_devices() && topo.world > 1)
                       .add("rccl_transport", tr.transport)
                       .add("rccl_nnodes", tr.nnodes)
                       .add("transport_verified", terr.empty()),
                true);
    }
  return 0;
}

}  // namespace

constexpr const char* kUsage =
    "usage: miint info\n"
    "       miint bench [--integrand pi4] [--n 1e9] [--dtype fp64|fp32|fp32acc] [--rule left]\n"
    "                   [--iters 200] [--gpus G] [--div series_exact|series|ieee] [--unfused] [--no-graph]\n"
    "                   [--block B] [--grid G] [--step-streams S] [--trig-library] [--settle N]\n"
    "                   [--no-multistep] [--slots K] [--close auto|kernel|launch] [--no-ar-host]\n"
    "                   [--diagnose]\n"
    "       miint sweep [--gpus G]\n"
    "       miint table2d [--grid 4096] [--gpus G] [--slice R/W] [--no-graph]\n"
    "                     [--step-streams S] [--min-wg W] [--settle-ms MS] [--no-multistep]\n"
    "                     [--phases P] [--graph-steps K]\n"
    "       miint selfcheck\n"
    "       miint comm [--gpus G] [--max-bytes 144e6] [--iters 20]\n"
    "Every record is one JSON line on stdout; --jsonl FILE also appends it to FILE.\n";

int main(int argc, char** argv) {
  try {
    cli::Args a(argc, argv);
    if (cli::usage_requested(a, kUsage)) return 0;
    const std::string cmd = a.positional().empty() ? "info" : a.positional()[0];
    if (cmd == "info") {
      const int nd = device_count();
      std::printf("miint: %d HIP device(s), RCCL %s\n", nd, nd ? RcclComm::version().c_str() : "-");
      for (int d = 0; d < nd; ++d) {
        const DeviceInfo i = device_info(d);
        std::printf("  [%d] %s %s  %d CUs  %.1f GHz  %.1f GB  L2 %d KB  LDS %zu KB/CU (%zu KB/block)\n",
                    d, i.name.c_str(), i.arch.c_str(), i.num_cus, i.clock_khz / 1e6,
                    i.total_mem / 1e9, i.l2_bytes / 1024, i.lds_per_cu / 1024,
                    i.lds_per_block / 1024);
      }
      return 0;
    }
    if (cmd == "selfcheck") return selfcheck();
    const cli::Topology topo = cli::topology(a);
    const int iters = static_cast<int>(a.integer("iters", 100));
    const bool graphs = !a.flag("no-graph");
    if (cmd == "bench") {
      RiemannConfig c = make_cfg(a.str("integrand", "pi4"), a.num("n", 1e9), a.str("dtype", "fp64"),
                                 a.str("rule", "left"), a.str("div", "series_exact"));
      c.fused = !a.flag("unfused");
      c.grid = static_cast<int>(a.integer("grid", 0));
      c.block = static_cast<int>(a.integer("block", kRiemannBlock));
      c.step_streams = static_cast<int>(a.integer("step-streams", 0));
      c.multistep = !a.flag("no-multistep");  // A-B: chained batches instead
      c.slots = static_cast<int>(a.integer("slots", c.slots));
      // A-B knobs of a multi-step batch's tail (profiles/r6/batch_tail.md): the closing
      // kernel or the in-launch close; the bucketed all-reduce into pinned host slots or
      // into the device buffer and a copy
      c.close = a.str("close", c.close);
      c.allreduce_to_host = !a.flag("no-ar-host");
      // validation / A-B: kIeee sin and cos by ocml per sample instead of fast_trig.hpp
      if (a.flag("trig-library")) set_trig_library(true);
      MIINT_CHECK(riemann_block_ok(c.block), "--block must be 64, 128, 256, 512 or 1024");
      c.waves_per_cu = static_cast<int>(a.integer("waves-per-cu", 32));
      // --settle N: untimed steps before the timed ones (default: ~60 ms worth; profiler
      // runs pass a few, so the trace holds little more than the timed dispatches)
      const BenchRow r = bench_one(topo, c, iters, graphs,
                                   static_cast<int>(a.integer("settle", -1)),
                                   a.flag("diagnose"));
      if (topo.rank0 == 0)
        print_row(a, r, a.str("integrand", "pi4").c_str(), a.str("dtype", "fp64").c_str(),
                  a.str("rule", "left").c_str());
      return 0;
    }
    if (cmd == "table2d") {  // BASELINE config #5: 2-D field, g x g samples, rows split
      Table2DConfig c;
      c.grid = static_cast<int>(a.integer("grid", 4096));
      c.bucket = !a.flag("no-bucket");  // one all-reduce per graph replay
      c.chain = !a.flag("no-chain");    // graph replays: chained launches, no per-launch tail
      c.step_streams = static_cast<int>(a.integer("step-streams", 0));  // chains per replay
      c.min_wg = static_cast<int>(a.integer("min-wg", 0));
      c.settle_ms = a.num("settle-ms", c.settle_ms);
      c.multistep = !a.flag("no-multistep");  // A-B: chained launches per integration
      c.phases = static_cast<int>(a.integer("phases", 0));  // multi-step step phases (0 auto)
      c.graph_steps = static_cast<int>(a.integer("graph-steps", 0));  // per replay (0 auto)
      // --slice R/W: time only rank R's rows of a W-GPU split, on this GPU (no collective)
      const std::string sl = a.str("slice", "");
      if (!sl.empty()) {
        const size_t k = sl.find('/');
        if (k == std::string::npos) fail("--slice wants R/W", __FILE__, __LINE__);
        c.rank = std::stoi(sl.substr(0, k));
        c.world = std::stoi(sl.substr(k + 1));
      }
      double value = 0.0, timed = 0.0, ms = 0.0;
      bool bucketed = false, chained = false, multistep = false;
      int streams = 1, phases = 0, resident = 0, min_wg = 0, wgs = 0, gsteps = 0;
      cli::RankFacts facts;
      std::mutex mu;
      cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
        Table2DPlan plan(c, dev, comm);
        RankAgree agree(comm);
        const double v = plan.run();
        const double t = agree.max(plan.time(iters, graphs));  // barrier inside; slowest rank
        std::lock_guard<std::mutex> g(mu);
        if (rank == topo.rank0) {
          facts.note(comm);
          value = v;
          timed = plan.last_result();
          bucketed = plan.bucketed() && graphs;
          chained = plan.chained() && graphs;
          multistep = plan.multistep() && graphs;
          streams = chained ? plan.step_streams() : 1;
          phases = multistep ? plan.phases() : 0;
          resident = plan.resident_per_cu();
          min_wg = plan.min_wg();
          wgs = plan.workgroups();
          gsteps = graphs ? plan.graph_steps() : 0;
        }
        if (t > ms) ms = t;
      });
      if (topo.rank0 == 0) {
        cli::JsonRecord r;
        r.add("program", "table2d").add("grid", c.grid);
        r.add("step_streams", streams).add("multistep", multistep).add("phases", phases);
        r.add("resident_per_cu", resident).add("min_wg", min_wg).add("workgroups", wgs);
        r.add("graph_steps", gsteps);
        facts.add(r, topo);
        if (c.world > 1) {
          r.add("slice", std::to_string(c.rank) + "/" + std::to_string(c.world))
              .add("partial", value);
        } else {
          const double want = table2d_oracle(c.grid);
          const double exact = 122000.004 * 122000.004;
          r.add("gpus", topo.world)
              .add("result", value)
              .add("timed_result", timed)
              .add("bucketed_allreduce", bucketed)
              .add("chained", chained)
              .add("midpoint_oracle", want)
              .add("rel_err_vs_oracle", std::fabs(value - want) / want)
              .add("rel_err_vs_exact", std::fabs(value - exact) / exact)
              .add("samples_per_s", static_cast<double>(c.grid) * c.grid / (ms * 1e-3));
        }
        cli::emit(a, r.add("ms_per_integration", ms), true);
      }
      return 0;
    }
    if (cmd == "comm") return comm_sweep(a, topo, a.num("max-bytes", 144e6), static_cast<int>(a.integer("iters", 20)));
    if (cmd == "sweep") {
      const std::vector<double> ns = {1e6, 1e9, 1e10};
      const std::vector<std::string> integs = {"pi4", "sin", "poly", "train"};
      for (const auto& integ : integs)
        for (const char* dt : {"fp64", "fp32"}) {
          if (std::string(dt) == "fp32" && integ != "pi4") continue;
          for (double n : ns) {
            if (integ != "pi4" && n > 1e9) continue;
            RiemannConfig c = make_cfg(integ, n, dt, "left", "series");
            const int it = n >= 1e10 ? 10 : (n >= 1e9 ? 50 : 500);
            const BenchRow r = bench_one(topo, c, it, graphs);
            if (topo.rank0 == 0) print_row(a, r, integ.c_str(), dt, "left");
          }
        }
      return 0;
    }
    std::fprintf(stderr, "usage: miint info|bench|sweep|table2d|comm|selfcheck [--flags]\n");
    return 2;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "miint: %s\n", e.what());
    return 1;
  }
}
