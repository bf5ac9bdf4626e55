// trainscan — distributed two-phase prefix scan of the train profile (reference: 4main.c).
//
// Output (4main.c:73,239,241):
//   Step size of 10000
//   %lf seconds
//   Total distance traveled = %lf
// Per GPU (default --algo fused): closed-form tile sums with in-block scans and a
// last-workgroup block scan, then one write pass that generates the samples again and stores
// both running integrals; across GPUs an allgather of one {T1, T2, count} triple per rank and
// on-device carries (no 144 MB gathers, no serial carry loop on a root, no broadcast).
// --algo lookback: one interp+scan kernel (decoupled look-back) per phase; onepass: a single
// look-back pass over the two-component tile state. --parity reproduces 4main's partitions and
// printed element (P=7 -> 0.000000, P=16 -> 117642.707174). --replicate allgathers the full
// table to every rank like 4main.c:157.
//
// --device cpu runs the pipeline on host threads (and host ranks under torchrun-style env):
// per-thread closed totals, an exclusive scan of the thread/rank totals, one compensated
// write pass of vel and pos (2 x 144 MB, as 4main.c materialises them; --no-keep forms the
// totals only); --parity there is the reference's sequential emulation for --ranks P.
//
//   ./trainscan [--gpus G] [--parity] [--replicate] [--no-phase2] [--algo onepass|fused|lookback]
//               [--steps-per-sec S] [--iters K] [--json] [--jsonl FILE]
//               [--device cpu [--threads T] [--ranks P] [--no-keep]] [--profile FILE]
#include <cmath>
#include <cstdio>

#include "cli_common.hpp"
#include "miint/host.hpp"
#include "miint/oracle.hpp"
#include "miint/trainscan.hpp"

using namespace miint;

namespace {

int run_host(const cli::Args& a) {
  cli::HostRanks hr = cli::host_ranks(a);
  HostPool pool(hr.threads);
  HostScanConfig c;
  c.steps_per_sec = static_cast<int>(a.integer("steps-per-sec", oracle::kStepsPerSec));
  if (a.has("profile")) {
    c.table = oracle::load_profile(a.str("profile", ""));
    c.seconds = static_cast<int>(c.table.size() - 1);
  }
  c.keep = !a.flag("no-keep");
  const int iters = static_cast<int>(a.integer("iters", 1));
  if (hr.rank == 0) std::printf("Step size of %ld\n", static_cast<long>(c.steps_per_sec));
  double distance = 0.0, sos = 0.0, best = 0.0;
  int ranks = hr.world;
  MIINT_CHECK(!(a.has("profile") && a.flag("parity")), "--parity emulates the built-in profile");
  if (a.flag("parity")) {  // 4main.c's partitions and sequential sums for --ranks P
    MIINT_CHECK(hr.world == 1 && c.steps_per_sec == oracle::kStepsPerSec,
                "--device cpu --parity emulates --ranks P of 4main.c in one process");
    ranks = static_cast<int>(a.integer("ranks", 1));
    const double t0 = wall_seconds();
    const oracle::TrainScanParity r = oracle::trainscan_parity(ranks);
    distance = r.distance;
    sos = r.sum_of_sums;
    best = (wall_seconds() - t0) * 1e3;
  } else {
    std::vector<double> vel, pos;  // this rank's slice, materialised like 4main.c's arrays
    for (int i = 0; i < iters; ++i) {  // best of --iters
      if (hr.comm) hr.comm->barrier();
      const HostScanResult r = host_trainscan(c, pool, hr.comm.get(), c.keep ? &vel : nullptr,
                                              c.keep ? &pos : nullptr);
      if (i == 0 || r.seconds * 1e3 < best) best = r.seconds * 1e3;
      distance = r.distance;
      sos = r.sum_of_sums;
    }
  }
  if (hr.rank != 0) return 0;
  const double secs = wall_seconds() - process_start_seconds();
  std::printf("%lf seconds\n", secs);
  std::printf("Total distance traveled = %lf\n", distance);
  cli::emit(a, cli::JsonRecord()
                   .add("program", "trainscan")
                   .add("device", "cpu")
                   .add("isa", host_isa())
                   .add("ranks", ranks)
                   .add("threads_per_rank", pool.threads())
                   .add("parity", a.flag("parity"))
                   .add("materialized", c.keep && !a.flag("parity"))
                   .add("distance", distance)
                   .add("sum_of_sums", sos)
                   .add("host_ms", best)
                   .add("seconds_wall", secs));
  return 0;
}

}  // namespace

constexpr const char* kUsage =
    "usage: trainscan [--gpus G] [--loopback W] [--algo fused|lookback|onepass] [--parity]\n"
    "                 [--replicate] [--no-phase2] [--steps-per-sec S] [--iters K]\n"
    "                 [--json] [--jsonl FILE] [--profile FILE]\n"
    "                 [--device cpu [--threads T] [--ranks P] [--no-keep]]\n"
    "Distributed two-phase prefix scan of the train profile (velocity, then position).\n";

int main(int argc, char** argv) {
  try {
    cli::Args a(argc, argv);
    if (cli::usage_requested(a, kUsage)) return 0;
    if (cli::on_cpu(a)) return run_host(a);
    const cli::Topology topo = cli::topology(a);
    TrainScanConfig cfg;
    cfg.steps_per_sec = static_cast<int>(a.integer("steps-per-sec", oracle::kStepsPerSec));
    if (a.has("profile")) {  // a velocity profile of one's own (CSV/text, 1 s spacing)
      cfg.table = oracle::load_profile(a.str("profile", ""));
      cfg.seconds = static_cast<int>(cfg.table.size() - 1);
    }
    cfg.parity = a.flag("parity");
    MIINT_CHECK(!(a.has("profile") && cfg.parity), "--parity emulates the built-in profile");
    cfg.replicate = a.flag("replicate");
    cfg.phase2 = !a.flag("no-phase2");
    const std::string algo = a.str("algo", "fused");
    MIINT_CHECK(algo == "onepass" || algo == "fused" || algo == "lookback",
                "--algo must be onepass|fused|lookback");
    cfg.algo = algo == "fused"      ? ScanAlgo::kFused
               : algo == "lookback" ? ScanAlgo::kLookback
                                    : ScanAlgo::kOnePass;
    const int iters = static_cast<int>(a.integer("iters", 1));
    if (topo.rank0 == 0)  // 4main.c:72-74 (tablelen/1800)
      std::printf("Step size of %ld\n", static_cast<long>(cfg.steps_per_sec));
    TrainScanResult res;
    std::string timeout_what;
    cli::RankFacts facts;
    ReplicaDigest digest;
    bool replicas_identical = true;
    std::mutex mu;
    cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
      TrainScan ts(cfg, dev, comm);
      RankAgree agree(comm);
      TrainScanResult r;
      try {
        // every run starts behind a collective barrier; a timeout on any rank is agreed over
        // the communicator and thrown on every rank together (TrainScan::run)
        r = ts.run();
        for (int i = 1; i < iters; ++i) {  // --iters K: report the best device time
          const TrainScanResult q = ts.run();
          if (q.device_ms < r.device_ms) r.device_ms = q.device_ms;
        }
      } catch (const ScanTimeout& e) {
        r = TrainScanResult{};
        r.distance = r.sum_of_sums = std::nan("");
        r.timeout = 1;
        r.timeout_ranks = e.ranks;
        std::lock_guard<std::mutex> lk(mu);
        timeout_what = e.what();
      }
      if (!r.timeout) r.device_ms = agree.max(r.device_ms);  // the slowest rank's time
      // --replicate (4main.c:157: every rank ends holding the whole table): fingerprint each
      // rank's copy; the hashes are gathered, so rank 0 can say whether all copies are equal
      ReplicaDigest dg;
      bool identical = true;
      if (cfg.replicate && !r.timeout) {
        dg = ts.replica_digest();
        const double hi = static_cast<double>(dg.hash >> 32), lo = static_cast<double>(dg.hash & 0xffffffffu);
        const std::vector<double> all = agree.gather({hi, lo});
        for (size_t q = 0; q + 1 < all.size(); q += 2)
          identical = identical && all[q] == hi && all[q + 1] == lo;
      }
      std::lock_guard<std::mutex> lk(mu);
      if (rank == topo.rank0) {
        res = r;
        facts.note(comm);
        digest = dg;
        replicas_identical = identical;
      }
      if (r.timeout) res.timeout = 1;
    });
    if (!timeout_what.empty()) std::fprintf(stderr, "trainscan: %s\n", timeout_what.c_str());
    // exit status 3 on every rank when any rank's scan timed out (agreed in TrainScan::run)
    if (topo.rank0 != 0) return res.timeout ? 3 : 0;
    const double secs = wall_seconds() - process_start_seconds();
    std::printf("%lf seconds\n", secs);
    std::printf("Total distance traveled = %lf\n", res.distance);
    cli::JsonRecord rec;
    rec.add("program", "trainscan").add("gpus", topo.world);
    facts.add(rec, topo);
    if (cfg.replicate) {
      char hex[24];
      std::snprintf(hex, sizeof hex, "%016llx", static_cast<unsigned long long>(digest.hash));
      std::string at = "[";
      for (int k = 0; k < 5; ++k) {
        char b[40];
        std::snprintf(b, sizeof b, "%s%.17g", k ? ", " : "", digest.at[k]);
        at += b;
      }
      rec.add("replicate", true)
          .add("replica_n", static_cast<double>(digest.n))
          .add("replica_hash", std::string(hex))
          .add("replica_sum", digest.sum)
          .add_raw("replica_at", at + "]")
          .add("replicas_identical", replicas_identical);
    }
    cli::emit(a, rec.add("distance", res.distance)
                     .add("sum_of_sums", res.sum_of_sums)
                     .add("device_ms", res.device_ms)
                     .add("seconds_device", res.device_ms * 1e-3)
                     .add("timeout", static_cast<unsigned>(res.timeout))
                     .add("timeout_ranks", res.timeout_ranks)
                     .add("seconds_wall", secs));
    return res.timeout ? 3 : 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "trainscan: %s\n", e.what());
    return 1;
  }
}
