// Rank agreement (barrier / gather / max / any over a communicator) and RCCL transport
// evidence (see miint/comm.hpp).
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>

#include "miint/comm.hpp"
#include "miint/trace.hpp"

namespace miint {

// ------------------------------------------------------------------ rank agreement
RankAgree::RankAgree(const Comm* comm, double timeout_s)
    : comm_(comm && comm->world() > 1 ? comm : nullptr), timeout_s_(timeout_s) {
  if (!comm_) return;
  DeviceGuard g(comm_->device());
  const size_t w = static_cast<size_t>(comm_->world());
  MIINT_HIP(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  MIINT_HIP(hipMalloc(&send_, kMaxValues * sizeof(double)));
  MIINT_HIP(hipMemset(send_, 0, kMaxValues * sizeof(double)));  // the barrier's operand
  MIINT_HIP(hipMalloc(&recv_, w * kMaxValues * sizeof(double)));
  MIINT_HIP(hipHostMalloc(reinterpret_cast<void**>(&host_), w * kMaxValues * sizeof(double),
                          hipHostMallocDefault));
}

RankAgree::~RankAgree() {
  if (!comm_) return;
  (void)hipSetDevice(comm_->device());
  if (s_) (void)hipStreamSynchronize(s_);
  if (host_) (void)hipHostFree(host_);
  if (recv_) (void)hipFree(recv_);
  if (send_) (void)hipFree(send_);
  if (s_) (void)hipStreamDestroy(s_);
}

void RankAgree::barrier() const {
  if (!comm_) return;
  DeviceGuard g(comm_->device());
  // an all-reduce completes on a rank only once every rank has contributed to it
  comm_->allreduce_sum(send_, recv_, 1, s_);
  wait_with_timeout(s_, timeout_s_, comm_);
}

std::vector<double> RankAgree::gather(const std::vector<double>& v) const {
  MIINT_CHECK(v.size() >= 1 && v.size() <= kMaxValues, "RankAgree::gather: 1..16 values per rank");
  if (!comm_) return v;
  DeviceGuard g(comm_->device());
  const size_t k = v.size(), w = static_cast<size_t>(comm_->world());
  MIINT_HIP(hipMemcpyAsync(send_, v.data(), k * sizeof(double), hipMemcpyHostToDevice, s_));
  comm_->allgather(send_, recv_, k, s_);
  MIINT_HIP(hipMemcpyAsync(host_, recv_, w * k * sizeof(double), hipMemcpyDeviceToHost, s_));
  wait_with_timeout(s_, timeout_s_, comm_);
  return std::vector<double>(host_, host_ + w * k);
}

double RankAgree::max(double v) const {
  double m = v;
  for (double x : gather({v})) m = x > m ? x : m;
  return m;
}
double RankAgree::min(double v) const {
  double m = v;
  for (double x : gather({v})) m = x < m ? x : m;
  return m;
}
bool RankAgree::any(bool v) const { return max(v ? 1.0 : 0.0) > 0.0; }

// ------------------------------------------------------------------ RCCL transport evidence
namespace {

// "P2P/IPC/read" -> "P2P/IPC", "NET/Socket/0" -> "NET/Socket", "SHM/direct/direct" ->
// "SHM/direct": the transport and its mechanism, without channel / device suffixes
std::string transport_name(const std::string& tok) {
  std::string out;
  int parts = 0;
  size_t i = 0;
  while (i < tok.size() && parts < 2) {
    size_t j = tok.find('/', i);
    if (j == std::string::npos) j = tok.size();
    const std::string part = tok.substr(i, j - i);
    const bool numeric = !part.empty() && part.find_first_not_of("0123456789") == std::string::npos;
    if (part.empty() || (parts > 0 && numeric)) break;
    out += (parts ? "/" : "") + part;
    ++parts;
    i = j + 1;
  }
  return out;
}

int int_after(const std::string& line, const char* key) {
  const size_t p = line.find(key);
  if (p == std::string::npos) return -1;
  return std::atoi(line.c_str() + p + std::strlen(key));
}

std::mutex g_log_mu;
std::string g_log_path;  // set once per process by capture_rccl_log
bool g_log_done = false;
bool g_log_ours = false;  // our file (deleted at exit) vs the user's NCCL_DEBUG_FILE
bool g_echo_warn = false;  // the user set NCCL_DEBUG below INFO: WARN lines go to stderr

void finish_log() {
  if (g_log_path.empty()) return;
  if (g_echo_warn) {  // what the user's level would have shown them on stderr
    std::ifstream f(g_log_path);
    std::string line;
    while (std::getline(f, line))
      if (line.find(" WARN ") != std::string::npos) std::fprintf(stderr, "%s\n", line.c_str());
  }
  const char* keep = std::getenv("MIINT_RCCL_LOG_KEEP");
  if (g_log_ours && !(keep && *keep && std::strcmp(keep, "0") != 0))
    std::remove(g_log_path.c_str());
}

// RCCL's NCCL_DEBUG_FILE substitutions: %h = hostname, %p = pid
std::string expand_debug_file(const std::string& pat) {
  std::string out;
  for (size_t i = 0; i < pat.size(); ++i) {
    if (pat[i] == '%' && i + 1 < pat.size() && (pat[i + 1] == 'h' || pat[i + 1] == 'p')) {
      if (pat[i + 1] == 'p') {
        out += std::to_string(static_cast<long>(::getpid()));
      } else {
        char host[256] = {0};
        ::gethostname(host, sizeof(host) - 1);
        out += host;
      }
      ++i;
    } else {
      out += pat[i];
    }
  }
  return out;
}

}  // namespace

RcclTransport parse_rccl_log(const std::string& text) {
  RcclTransport t;
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    const size_t via = line.find(" via ");
    if (via != std::string::npos) {
      size_t b = via + 5, e = line.find_first_of(" \t\r", b);
      const std::string name = transport_name(line.substr(b, e == std::string::npos ? e : e - b));
      if (!name.empty()) {
        ++t.connections;
        // distinct names, first-seen order
        bool seen = false;
        size_t p = 0;
        while (p <= t.transport.size()) {
          size_t q = t.transport.find('+', p);
          if (q == std::string::npos) q = t.transport.size();
          if (t.transport.compare(p, q - p, name) == 0 && q - p == name.size()) seen = true;
          p = q + 1;
        }
        if (!seen) t.transport += (t.transport.empty() ? "" : "+") + name;
      }
    }
    const int nr = int_after(line, "nRanks ");
    if (nr > 0) {
      const int nn = int_after(line, "nNodes ");
      const int lr = int_after(line, "localRanks ");
      if (nr >= t.nranks) {
        t.nranks = nr;
        if (nn > 0) t.nnodes = nn;
        if (lr > 0) t.local_ranks = lr;
      }
    }
    if (line.find("Init COMPLETE") != std::string::npos) ++t.comms;
  }
  return t;
}

void capture_rccl_log() {
  std::lock_guard<std::mutex> g(g_log_mu);
  if (g_log_done) return;
  g_log_done = true;
  const char* off = std::getenv("MIINT_RCCL_LOG");
  if (off && std::strcmp(off, "0") == 0) return;
  const char* user_file = std::getenv("NCCL_DEBUG_FILE");
  const char* lvl = std::getenv("NCCL_DEBUG");
  const bool info = lvl && (std::strcmp(lvl, "INFO") == 0 || std::strcmp(lvl, "TRACE") == 0);
  if (user_file && *user_file) {
    // the user's file: read it, never overwrite or delete it. Without a level of their own
    // RCCL would write nothing into it, so INFO (INIT lines) is added in that case only.
    g_log_path = expand_debug_file(user_file);
    g_log_ours = false;
    if (!lvl || !*lvl) ::setenv("NCCL_DEBUG", "INFO", 1);
  } else {
    const char* tmp = std::getenv("TMPDIR");
    g_log_path = std::string(tmp && *tmp ? tmp : "/tmp") + "/miint_rccl." +
                 std::to_string(static_cast<long>(::getpid())) + ".log";
    std::remove(g_log_path.c_str());  // a stale file of a recycled pid
    g_log_ours = true;
    ::setenv("NCCL_DEBUG_FILE", g_log_path.c_str(), 1);
    // INFO lines of the INIT subsystem (comm topology + one line per peer connection) into
    // the file. A level the user chose below INFO (WARN, VERSION) loses nothing: its WARN
    // lines are echoed to stderr at exit.
    g_echo_warn = lvl && *lvl && !info;
    if (!info) ::setenv("NCCL_DEBUG", "INFO", 1);
  }
  const char* sub = std::getenv("NCCL_DEBUG_SUBSYS");
  if (!sub || !*sub) {
    // the peer-connection lines ("... via P2P/IPC") are INIT|P2P / INIT|NET messages; GRAPH
    // adds the topology search's channel lines ("Pattern .., nChannels ..", "Ring 00 : ..",
    // bench.py's diagnostic record) — all printed once per communicator, never per call
    ::setenv("NCCL_DEBUG_SUBSYS", "INIT,P2P,GRAPH", 1);
  } else if (sub[0] != '^' && !std::strstr(sub, "INIT") && !std::strstr(sub, "ALL")) {
    ::setenv("NCCL_DEBUG_SUBSYS", (std::string(sub) + ",INIT").c_str(), 1);
  }
  std::atexit(finish_log);
}

std::string transport_error(const RcclTransport& t, int world, int local_world, bool share) {
  if (world <= 1 || share || local_world != world) return "";
  if (t.transport.empty())
    return "RCCL transport unknown between " + std::to_string(world) +
           " ranks on distinct local GPUs (no peer connection in " +
           (t.log.empty() ? std::string("no RCCL log captured") : t.log) +
           "): P2P over xGMI cannot be confirmed";
  // every connection P2P: a network transport or shared host memory (SHM: P2P disabled) is
  // not xGMI
  bool all_p2p = true;
  for (size_t p = 0; p <= t.transport.size();) {
    size_t q = t.transport.find('+', p);
    if (q == std::string::npos) q = t.transport.size();
    all_p2p = all_p2p && t.transport.compare(p, 3, "P2P") == 0 && q - p >= 3;
    p = q + 1;
  }
  if (t.uses_net() || !all_p2p)
    return "RCCL transport is " + t.transport + " (nNodes " + std::to_string(t.nnodes) +
           ") between " + std::to_string(world) +
           " ranks on distinct local GPUs: expected P2P over xGMI";
  if (t.nnodes > 1)
    return "RCCL counted " + std::to_string(t.nnodes) + " nodes for " + std::to_string(world) +
           " ranks of one node";
  return "";
}

std::string rccl_log_path() {
  std::lock_guard<std::mutex> g(g_log_mu);
  return g_log_path;
}

RcclTransport rccl_transport() {
  const std::string path = rccl_log_path();
  if (path.empty()) return {};
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  RcclTransport t = parse_rccl_log(ss.str());
  t.log = path;
  return t;
}

}  // namespace miint
