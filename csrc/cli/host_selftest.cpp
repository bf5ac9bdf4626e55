// host_selftest — host-only checks of the native runtime's CPU side, built with
// AddressSanitizer + UndefinedBehaviorSanitizer (`make sanitize`).
//
// The reference ships latent host UB (uninitialised sums B1/B2, strlen of an
// uninitialised buffer B12, 288 MB of stack arrays B11, int overflow B9). The GPU-side
// sanitizers are not available on the target pool, so this binary exercises every host
// code path that needs no device — profile generation, oracles, parity emulation of all
// three reference programs, 64-bit slicing, CLI argument parsing, run records, the TCP
// rendezvous of the native multi-process launch, the host engine (thread pool, vector
// kernels, TCP host collectives, threaded train scan) — under ASan/UBSan.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "cli_common.hpp"
#include <unistd.h>

#include "miint/comm.hpp"
#include "miint/host.hpp"
#include "miint/integrator.hpp"
#include "miint/oracle.hpp"

using namespace miint;

static int g_bad = 0;
static void expect(bool ok, const char* what) {
  std::printf("%-60s %s\n", what, ok ? "ok" : "FAIL");
  g_bad += !ok;
}

int main() {
  const auto& v = oracle::profile_table();
  expect(v.size() == 1801 && v[0] == 0.0, "profile: 1801 entries, starts at rest");
  expect(std::fabs(oracle::profile_exact_integral() - 122000.004) < 1e-6, "profile integral");
  expect(std::fabs(oracle::interp(v, 400.5) - 87.14286) < 1e-9, "interp in cruise");
  expect(oracle::interp(v, 1800.0) == v[1800], "interp clamps at t = 1800 (B4 fixed)");

  char buf[32];
  std::snprintf(buf, sizeof buf, "%f", oracle::cintegrate_parity(32, 2));
  expect(std::string(buf) == "121999.800663", "cintegrate parity SP=32 SM=2");
  expect(oracle::trainscan_parity(7).distance == 0.0, "4main parity P=7 -> 0 (B13)");
  std::snprintf(buf, sizeof buf, "%f", oracle::trainscan_parity(16).distance);
  expect(std::string(buf) == "117642.707174", "4main parity P=16");
  expect(oracle::riemann_mpi_parity(1, 1e6) == 0.0, "riemann parity P=1 -> 0 (B10)");
  expect(std::fabs(oracle::riemann_mpi_parity(8, 1e6) - 2.0) < 1e-10, "riemann parity P=8");

  const long double pi4 =
      oracle::riemann_serial(Integrand::kPi4, 0.0, 1.0, 1000000, Rule::kLeft);
  expect(std::fabs(static_cast<double>(pi4) - M_PI - 1e-6) < 1e-9, "serial pi4 left N=1e6");

  // 64-bit slicing: exact cover, no dropped remainder (B5/B9/B13 fixed)
  const uint64_t n = (uint64_t(1) << 40) + 12345;
  uint64_t pos = 0;
  bool cover = true;
  for (int r = 0; r < 7; ++r) {
    uint64_t b, c;
    rank_slice(n, r, 7, &b, &c);
    cover &= (b == pos);
    pos += c;
  }
  expect(cover && pos == n, "rank_slice covers 2^40+12345 exactly");

  const char* argv[] = {"x", "pos", "--n", "1e10", "--gpus=4", "--parity"};
  cli::Args a(6, const_cast<char**>(argv));
  expect(a.integer("n", 0) == 10000000000LL && a.integer("gpus", 1) == 4 && a.flag("parity") &&
             a.positional().size() == 1,
         "cli argument parsing");

  bool threw = false;
  try {
    (void)cli::parse_integrand("bogus");
  } catch (const Error&) {
    threw = true;
  }
  expect(threw && cli::parse_integrand("pi") == Integrand::kPi4 &&
             cli::parse_integrand("table") == Integrand::kTable,
         "integrand names: aliases accepted, unknown names rejected");

  // run records: escaping, non-finite values, --jsonl appends
  const std::string path = "/tmp/miint_selftest_" + std::to_string(::getpid()) + ".jsonl";
  const std::string jl = "--jsonl=" + path;
  const char* argv2[] = {"x", jl.c_str()};
  cli::Args b(2, const_cast<char**>(argv2));
  cli::JsonRecord r;
  r.add("s", "a\"b\\c").add("x", 0.1).add("inf", INFINITY).add("i", 7).add("t", true);
  expect(r.str() == "{\"s\":\"a\\\"b\\\\c\",\"x\":0.10000000000000001,\"inf\":null,\"i\":7,"
                    "\"t\":true}",
         "json record: escapes, %.17g, non-finite -> null");
  cli::emit(b, r);
  cli::emit(b, cli::JsonRecord().add("k", 2));
  std::ifstream in(path);
  std::string l1, l2, l3;
  std::getline(in, l1);
  std::getline(in, l2);
  expect(l1.rfind("{\"s\":", 0) == 0 && l2.rfind("{\"k\":2,\"time_unix\":", 0) == 0 &&
             !std::getline(in, l3),
         "--jsonl appends one line per record");
  std::remove(path.c_str());

  // TCP rendezvous transport (the RCCL id itself needs a GPU with this RCCL): 4 ranks as
  // threads, rank 0 last to start, all receive rank 0's 128 bytes, zero bytes included
  std::string id(128, '\0');
  for (size_t k = 0; k < id.size(); ++k) id[k] = static_cast<char>(k * 37 + 11);
  std::vector<std::string> ids(4);
  std::vector<std::thread> th;
  const int port = 20000 + ::getpid() % 20000;
  for (int k = 3; k >= 0; --k)
    th.emplace_back([&, k] {
      ids[k] = rendezvous_share("127.0.0.1", port, k, 4, k == 0 ? id : std::string(), 128, 30.0);
    });
  for (auto& t : th) t.join();
  expect(ids[0] == id && ids[1] == id && ids[2] == id && ids[3] == id,
         "rendezvous: 4 ranks receive rank 0's 128-byte payload");
  bool timed_out = false;
  try {
    (void)rendezvous_share("127.0.0.1", port + 1, 1, 2, std::string(), 128, 0.2);
  } catch (const Error&) {
    timed_out = true;
  }
  expect(timed_out, "rendezvous: a rank whose rank 0 never listens times out");

  // host engine (miint/host.hpp): vector kernels on a thread pool, the threaded reference
  // program, the train scan with carries across 3 host ranks over the TCP star
  {
    HostPool pool(3);
    RiemannConfig c;
    c.integrand = Integrand::kSin;
    c.b = M_PI;
    c.n = 1000003;
    c.rule = Rule::kMid;
    expect(std::fabs(host_riemann(c, 0, c.n, pool) - 2.0) < 1e-12, "host engine: sin mid N=1e6+3");
    c.integrand = Integrand::kTable;
    c.b = 1800.0;
    c.n = 18000000 / 64;
    c.rule = Rule::kLeft;
    expect(std::fabs(host_riemann(c, 0, c.n, pool) - 122000.004) < 1e-3, "host engine: table");
    expect(host_riemann_mpi_parity(8, 1e6, M_PI, pool) == oracle::riemann_mpi_parity(8, 1e6),
           "host engine: threaded riemann.cpp == serial parity oracle");
    HostScanConfig sc;
    sc.seconds = 30;
    sc.keep = true;
    const HostScanResult one = host_trainscan(sc, pool, nullptr);
    std::vector<HostScanResult> rs(3);
    std::vector<std::vector<double>> vel(3), posv(3);
    std::vector<std::thread> hr;
    const int hport = 20000 + (::getpid() + 7919) % 20000;
    for (int k = 2; k >= 0; --k)
      hr.emplace_back([&, k] {
        HostComm comm("127.0.0.1", hport, k, 3, 30.0);
        HostPool p2(2);
        rs[k] = host_trainscan(sc, p2, &comm, &vel[k], &posv[k]);
      });
    for (auto& t : hr) t.join();
    expect(std::fabs(rs[0].distance - one.distance) < 1e-9 * one.distance &&
               rs[2].distance == rs[0].distance && vel[2].size() == rs[2].count &&
               std::fabs(vel[2].back() / sc.steps_per_sec - one.distance) < 1e-9 * one.distance,
           "host engine: train scan over 3 ranks (TCP star) == one rank");
  }

  std::printf("%s\n", g_bad ? "HOST SELFTEST FAILED" : "HOST SELFTEST OK");
  return g_bad ? 1 : 0;
}
