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
//   ./trainscan [--gpus G] [--parity] [--replicate] [--no-phase2] [--algo onepass|fused|lookback]
//               [--steps-per-sec S] [--iters K] [--json] [--jsonl FILE]
#include <cstdio>

#include "cli_common.hpp"
#include "miint/oracle.hpp"
#include "miint/trainscan.hpp"

using namespace miint;

int main(int argc, char** argv) {
  try {
    cli::Args a(argc, argv);
    const cli::Topology topo = cli::topology(a);
    TrainScanConfig cfg;
    cfg.steps_per_sec = static_cast<int>(a.integer("steps-per-sec", oracle::kStepsPerSec));
    cfg.parity = a.flag("parity");
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
    std::mutex mu;
    cli::run_ranks(topo, [&](int rank, int dev, const Comm* comm) {
      TrainScan ts(cfg, dev, comm);
      TrainScanResult r = ts.run();
      for (int i = 1; i < iters; ++i) {  // --iters K: report the best device time
        const TrainScanResult q = ts.run();
        if (q.device_ms < r.device_ms) r.device_ms = q.device_ms;
        r.timeout |= q.timeout;
      }
      std::lock_guard<std::mutex> lk(mu);
      if (rank == topo.rank0) res = r;
    });
    if (topo.rank0 != 0) return 0;
    const double secs = wall_seconds() - process_start_seconds();
    std::printf("%lf seconds\n", secs);
    std::printf("Total distance traveled = %lf\n", res.distance);
    cli::emit(a, cli::JsonRecord()
                     .add("program", "trainscan")
                     .add("gpus", topo.world)
                     .add("distance", res.distance)
                     .add("sum_of_sums", res.sum_of_sums)
                     .add("device_ms", res.device_ms)
                     .add("seconds_device", res.device_ms * 1e-3)
                     .add("timeout", static_cast<unsigned>(res.timeout))
                     .add("seconds_wall", secs));
    return res.timeout ? 3 : 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "trainscan: %s\n", e.what());
    return 1;
  }
}
