// Shared plumbing for the miint command-line tools.
//
// The reference takes no arguments at all (every knob is a #define, SURVEY §5 "Config /
// flags"); these tools default to the reference's configuration and expose the rest as
// --flags. Launch topologies (replacing `mpirun -np P`):
//   * one process driving G GPUs:      ./riemann --gpus 8          (ncclCommInitAll + threads)
//   * one process per GPU via torchrun: torchrun --no-python --nproc-per-node 8 ./riemann
//     (RANK/WORLD_SIZE/LOCAL_RANK from the env, RCCL unique id over a TCP rendezvous on
//     MASTER_ADDR:MASTER_PORT+17)
//   * W logical ranks on one GPU:      ./riemann --loopback 8   (LoopbackComm, threads;
//     exercises every world > 1 path on a one-GPU box)
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "miint/comm.hpp"
#include "miint/host.hpp"
#include "miint/runtime.hpp"

namespace miint {
namespace cli {

class Args {
 public:
  Args(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.rfind("--", 0) != 0) { pos_.push_back(a); continue; }
      a = a.substr(2);
      const auto eq = a.find('=');
      if (eq != std::string::npos) kv_[a.substr(0, eq)] = a.substr(eq + 1);
      else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) kv_[a] = argv[++i];
      else kv_[a] = "1";
    }
  }
  bool has(const std::string& k) const { return kv_.count(k) > 0; }
  std::string str(const std::string& k, const std::string& d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : it->second;
  }
  double num(const std::string& k, double d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : std::strtod(it->second.c_str(), nullptr);
  }
  long long integer(const std::string& k, long long d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : static_cast<long long>(std::strtod(it->second.c_str(), nullptr));
  }
  bool flag(const std::string& k) const {
    auto it = kv_.find(k);
    return it != kv_.end() && it->second != "0" && it->second != "false";
  }
  const std::vector<std::string>& positional() const { return pos_; }
  // --help / -h: the caller prints its usage text and exits before touching any device
  bool help() const {
    return kv_.count("help") > 0 || std::find(pos_.begin(), pos_.end(), "-h") != pos_.end();
  }

 private:
  std::map<std::string, std::string> kv_;
  std::vector<std::string> pos_;
};

// Strict spellings of the shared knobs: a typo fails instead of running the default.
inline DType parse_dtype(const std::string& s) {
  if (s == "fp64") return DType::kF64;
  if (s == "fp32") return DType::kF32;
  if (s == "fp32acc") return DType::kF32Acc32;
  fail("--dtype must be fp64, fp32 or fp32acc (got " + s + ")", __FILE__, __LINE__);
}
inline Rule parse_rule(const std::string& s) {
  if (s == "left") return Rule::kLeft;
  if (s == "mid") return Rule::kMid;
  if (s == "right") return Rule::kRight;
  fail("--rule must be left, mid or right (got " + s + ")", __FILE__, __LINE__);
}
inline DivMode parse_div(const std::string& s) {
  if (s == "series") return DivMode::kSeries;
  if (s == "ieee") return DivMode::kIeee;
  if (s == "series_exact") return DivMode::kSeriesExact;
  fail("--div must be series, series_exact or ieee (got " + s + ")", __FILE__, __LINE__);
}

// Print `text` and return true when --help / -h was given (main returns 0 then).
inline bool usage_requested(const Args& a, const char* text) {
  if (!a.help()) return false;
  std::fputs(text, stdout);
  return true;
}

inline int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : d;
}

struct Topology {
  int world = 1;        // total ranks (GPUs)
  int rank0 = 0;        // first rank handled by this process
  int local = 1;        // ranks (threads) in this process
  bool multiproc = false;
  bool loopback = false;  // --loopback W: W logical ranks on device 0 (LoopbackComm)
};

// Decide who runs what: torchrun env -> one rank per process; else --gpus threads.
inline Topology topology(const Args& a) {
  Topology t;
  const int ws = env_int("WORLD_SIZE", 1);
  if (a.has("loopback")) {
    // every multi-rank code path (slicing, collectives, group graphs, parity windows) with
    // W ranks on the one GPU of the test pool; not a performance configuration
    t.world = static_cast<int>(a.integer("loopback", 2));
    MIINT_CHECK(t.world >= 1 && t.world <= kMaxLoopbackRanks, "--loopback W needs 1 <= W <= 16");
    MIINT_CHECK(ws == 1, "--loopback runs in one process (no torchrun)");
    MIINT_CHECK(device_count() >= 1, "--loopback needs a HIP device (no HIP devices visible)");
    t.local = t.world;
    t.loopback = true;
    return t;
  }
  if (ws > 1) {
    t.world = ws;
    t.rank0 = env_int("RANK", 0);
    t.local = 1;
    t.multiproc = true;
  } else {
    t.world = static_cast<int>(a.integer("gpus", 1));
    if (t.world < 1) t.world = 1;
    const int nd = device_count();
    if (nd < t.world) fail("--gpus " + std::to_string(t.world) + " but only " +
                           std::to_string(nd) + " HIP devices visible", __FILE__, __LINE__);
    t.local = t.world;
  }
  return t;
}

// Run fn(rank, device, comm) for every rank this process owns (threads when > 1) and
// rethrow the first failure. comm is null when world == 1.
inline void run_ranks(const Topology& t,
                      const std::function<void(int rank, int device, const Comm* comm)>& fn) {
  std::vector<std::unique_ptr<Comm>> comms;
  if (!t.loopback && t.world > 1) capture_rccl_log();  // transport evidence for the record
  if (t.loopback) {
    run_loopback(t.world, 0, [&](int r, const Comm* c) { fn(r, 0, t.world > 1 ? c : nullptr); });
    return;
  }
  if (t.multiproc) {
    const char* addr = std::getenv("MASTER_ADDR");
    const int port = env_int("MASTER_PORT", 29500) + 17;
    const std::string id = rendezvous_unique_id(addr ? addr : "127.0.0.1", port, t.rank0, t.world);
    const int dev = rank_device(env_int("LOCAL_RANK", 0));
    comms.emplace_back(new RcclComm(id, t.rank0, t.world, dev));
    fn(t.rank0, dev, comms[0].get());
    return;
  }
  if (t.world == 1) {
    fn(0, 0, nullptr);
    return;
  }
  std::vector<int> devs(t.world);
  for (int i = 0; i < t.world; ++i) devs[i] = i;
  comms = RcclComm::init_all(devs);
  std::vector<std::thread> th;
  std::mutex mu;
  std::string err;
  for (int r = 0; r < t.world; ++r) {
    th.emplace_back([&, r] {
      try {
        fn(r, r, comms[r].get());
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        if (err.empty()) err = "rank " + std::to_string(r) + ": " + e.what();
      }
    });
  }
  for (auto& x : th) x.join();
  if (!err.empty()) throw Error(err);
}

// --device cpu: the reference's MPI side on this host (riemann.cpp / 4main.c are CPU
// programs). Ranks are processes — under torchrun-style env (WORLD_SIZE, RANK,
// LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT; host collectives on MASTER_PORT + 19) — or
// this one process; each rank runs --threads T workers (default: the cores shared among the
// node's ranks). No HIP call is made on this path, so it runs on a GPU-less box.
inline bool on_cpu(const Args& a) {
  const std::string d = a.str("device", "gpu");
  MIINT_CHECK(d == "gpu" || d == "cpu", "--device must be gpu|cpu");
  return d == "cpu";
}
struct HostRanks {
  int rank = 0, world = 1, threads = 1;
  std::unique_ptr<HostComm> comm;  // world > 1
};
inline HostRanks host_ranks(const Args& a) {
  HostRanks h;
  h.world = env_int("WORLD_SIZE", 1);
  h.rank = env_int("RANK", 0);
  const int local = std::max(1, env_int("LOCAL_WORLD_SIZE", h.world));
  // --threads, else the node's host threads (HostPool's default: MIINT_HOST_THREADS /
  // OMP_NUM_THREADS / affinity) shared among the node's ranks
  h.threads = static_cast<int>(a.integer("threads", 0));
  if (h.threads <= 0) h.threads = std::max(1, HostPool::default_threads() / local);
  if (h.world > 1) {
    const char* addr = std::getenv("MASTER_ADDR");
    h.comm.reset(new HostComm(addr ? addr : "127.0.0.1", env_int("MASTER_PORT", 29500) + 19,
                              h.rank, h.world));
  }
  return h;
}

// --integrand names shared by every tool (SURVEY §5 config flags); unknown names fail.
inline Integrand parse_integrand(const std::string& s) {
  if (s == "sin") return Integrand::kSin;
  if (s == "pi4" || s == "pi") return Integrand::kPi4;
  if (s == "poly") return Integrand::kPoly;
  if (s == "train") return Integrand::kTrainVel;
  if (s == "table") return Integrand::kTable;
  if (s == "table2d") fail("the 2-D field is its own tool: miint table2d [--grid 4096]", __FILE__, __LINE__);
  fail("unknown integrand '" + s + "' (sin|pi4|poly|train|table)", __FILE__, __LINE__);
}

inline std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o;
}

// One flat JSON object, keys in insertion order (SURVEY §5 "Metrics / logging": the run
// record of every tool). Doubles print round-trippable (%.17g); non-finite ones as null.
class JsonRecord {
 public:
  JsonRecord& add(const std::string& k, double v) {
    char b[40];
    if (std::isfinite(v)) std::snprintf(b, sizeof b, "%.17g", v);
    else std::snprintf(b, sizeof b, "null");
    return raw(k, b);
  }
  JsonRecord& add(const std::string& k, int v) { return raw(k, std::to_string(v)); }
  JsonRecord& add(const std::string& k, unsigned v) { return raw(k, std::to_string(v)); }
  JsonRecord& add(const std::string& k, bool v) { return raw(k, v ? "true" : "false"); }
  JsonRecord& add(const std::string& k, const std::string& v) {
    return raw(k, "\"" + json_escape(v) + "\"");
  }
  JsonRecord& add(const std::string& k, const char* v) { return add(k, std::string(v)); }
  // a value that is already JSON (an array, a nested object)
  JsonRecord& add_raw(const std::string& k, const std::string& json) { return raw(k, json); }
  std::string str() const { return "{" + body_ + "}"; }

 private:
  JsonRecord& raw(const std::string& k, const std::string& v) {
    if (!body_.empty()) body_ += ",";
    body_ += "\"" + json_escape(k) + "\":" + v;
    return *this;
  }
  std::string body_;
};

// --json prints the record on stdout after the reference's lines; --jsonl PATH appends it
// to PATH (one object per line; the results log the SURVEY §5 checkpoint row asks for, so
// sweeps across launches accumulate in one file). Both may be given. Tools whose output IS
// the record (miint) pass print = true.
inline void emit(const Args& a, JsonRecord r, bool print = false) {
  r.add("time_unix", static_cast<double>(std::time(nullptr)));
  const std::string line = r.str();
  if (print || a.flag("json")) {
    std::printf("%s\n", line.c_str());
    std::fflush(stdout);
  }
  const std::string path = a.str("jsonl", "");
  if (!path.empty()) {
    std::FILE* f = std::fopen(path.c_str(), "a");
    if (!f) fail("--jsonl: cannot open " + path + " for appending", __FILE__, __LINE__);
    std::fprintf(f, "%s\n", line.c_str());
    std::fclose(f);
  }
}

// What a multi-rank record says about its ranks (the records must show how the
// ranks met). Filled by the rank that prints (note()), added by add().
struct RankFacts {
  std::string comm = "none";  // communicator kind: rccl | loopback | none (one rank)
  int rccl_world = 0;         // ranks the transport reports (ncclCommCount); 0 without RCCL
  void note(const Comm* c) {
    if (!c) return;
    comm = c->kind();
    if (comm == "rccl") rccl_world = c->transport_world();
  }
  // ranks_share_gpus: MIINT_OVERSUBSCRIBE (W ranks on fewer GPUs, RCCL over loopback
  // sockets): a correctness run of the multi-rank path, never a performance number.
  // rccl_transport / rccl_nnodes: what RCCL's INIT log says the connections use.
  void add(JsonRecord& r, const Topology& t) const {
    r.add("comm", comm).add("ranks_share_gpus", ranks_share_devices() && t.world > 1);
    r.add("rccl_world", rccl_world);
    const RcclTransport tr = rccl_world > 0 ? rccl_transport() : RcclTransport{};
    r.add("rccl_transport", tr.transport).add("rccl_nnodes", tr.nnodes);
    // fail-closed: RCCL ranks of one node on distinct GPUs must be SEEN meeting
    // over P2P/xGMI; no evidence, sockets or a multi-node count is recorded as an error
    std::string err;
    if (comm == "rccl") {
      const int local_world = t.multiproc ? env_int("LOCAL_WORLD_SIZE", t.world) : t.world;
      err = transport_error(tr, t.world, local_world, ranks_share_devices() && t.world > 1);
      if (!err.empty()) std::fprintf(stderr, "transport check: %s\n", err.c_str());
    }
    r.add("transport_verified", err.empty());
    if (!err.empty()) r.add("transport_error", err);
  }
};

// Median of a sample (host timings).
inline double median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

}  // namespace cli
}  // namespace miint
