// Communicators: the collectives every multi-rank plan runs on a stream.
//
// Replaces every MPI call site of the reference:
//   riemann.cpp:76,82-85   worker MPI_Send + root MPI_Recv loop  -> allreduce_sum(1 x f64)
//   4main.c:134,200        MPI_Reduce of local sums              -> allreduce_sum
//   4main.c:141-157        slice gather to root + serial carry + 144 MB Bcast
//                          -> allgather of P block totals (P x 8 B) + on-device carry add;
//                             optional allgather of the full table when every rank needs it
//   4main.c:137 Barrier    -> stream order (or a 0-byte-equivalent allreduce)
//
// `Comm` is the interface the plans (RiemannPlan, TrainScan, Table2DPlan) program against:
// stream-ordered fp64 collectives plus two graph hooks (capture / launch), because how a
// batch of steps that contains collectives becomes a hipGraph depends on the transport.
//
//   RcclComm      production: RCCL over xGMI, one rank per GPU. Two bootstraps: one process
//                 per GPU (unique id shared out of band: torch.distributed's store or miint's
//                 TCP rendezvous) and one process driving every GPU (ncclCommInitAll).
//                 Collectives are RCCL kernels on the caller's stream, so a rank's graph
//                 simply captures them.
//   LoopbackComm  W logical ranks on ONE device, one host thread per rank (test transport:
//                 the gpurun pool has one GPU and RCCL refuses two ranks on a device). Every
//                 collective is a host barrier at ENQUEUE time plus cross-stream events, a
//                 fixed-rank-order sum kernel and device copies, all stream-ordered; nothing
//                 spins on the device, and every event a stream waits on was recorded before
//                 the wait was enqueued, so no interleaving of the ranks' streams on the
//                 hardware queues can deadlock. Graph capture is group-wide: rank 0 opens one
//                 capture on a group stream and every rank enqueues its batch onto THAT
//                 stream (HIP calls serialised, the collectives' barriers order the ranks'
//                 work), so the W ranks' batches, collectives included, become ONE graph,
//                 launched once per batch for the whole group. (Ranks capturing on their own
//                 streams joined by cross-stream event waits crash the ROCm 7.0 runtime that
//                 PyTorch bundles, and need no more coverage than this: the per-rank stream
//                 choreography is what the direct, uncaptured path exercises.)
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "miint/common.hpp"
#include "miint/runtime.hpp"

#define MIINT_RCCL(expr)                                                                 \
  do {                                                                                   \
    ncclResult_t miint_r_ = (expr);                                                      \
    if (miint_r_ != ncclSuccess)                                                         \
      ::miint::fail(std::string(#expr) + " -> " + ncclGetErrorString(miint_r_), __FILE__, \
                    __LINE__);                                                           \
  } while (0)

namespace miint {

class Comm {
 public:
  virtual ~Comm() = default;
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  virtual const char* kind() const = 0;
  // Ranks the transport itself reports (ncclCommCount for RCCL): what the collectives
  // actually span, independent of how the launcher counted processes.
  virtual int transport_world() const = 0;

  virtual void allreduce_sum(const double* send, double* recv, size_t count,
                             hipStream_t s) const = 0;
  // recv holds world x count_per_rank values in rank order.
  virtual void allgather(const double* send, double* recv, size_t count_per_rank,
                         hipStream_t s) const = 0;
  virtual void broadcast(double* buf, size_t count, int root, hipStream_t s) const = 0;
  virtual void reduce_sum(const double* send, double* recv, size_t count, int root,
                          hipStream_t s) const = 0;
  // Throws if the transport reported an asynchronous error (e.g. a peer died).
  virtual void check_async() const {}
  // Abort outstanding collectives (watchdog path); the communicator is unusable afterwards.
  virtual void abort() const {}

  // Capture everything `body` enqueues on `s` into `g` / replay it. Every rank of a
  // communicator calls these collectively (same order, same batches).
  virtual void capture(Graph& g, hipStream_t s,
                       const std::function<void(hipStream_t)>& body) const {
    g.capture(s, body);
  }
  virtual void launch(const Graph& g, hipStream_t s) const { g.launch(s); }
  // True if capture() hands its body ONE stream shared by the whole group: the body must
  // then enqueue everything on that stream (no fork/join onto side streams).
  virtual bool capture_single_stream() const { return false; }

 protected:
  Comm(int rank, int world, int device) : rank_(rank), world_(world), device_(device) {}
  int rank_ = 0, world_ = 1, device_ = 0;
};

// Capture / launch through `comm` when there is one (group-wide graphs), else plainly.
inline void capture_with(const Comm* comm, Graph& g, hipStream_t s,
                         const std::function<void(hipStream_t)>& body) {
  if (comm) comm->capture(g, s, body);
  else g.capture(s, body);
}
inline void launch_with(const Comm* comm, const Graph& g, hipStream_t s) {
  if (comm) comm->launch(g, s);
  else g.launch(s);
}

// Ranks that share a GPU (MIINT_OVERSUBSCRIBE=1: more ranks than devices, e.g. W ranks on
// the one GPU of a test box). RCCL refuses two ranks of one host on one device ("Duplicate
// GPU detected"), so each such rank presents itself as a host of its own (NCCL_HOSTID) and
// the ranks meet over RCCL's socket transport on loopback (NCCL_SOCKET_IFNAME=lo unless set).
// The multi-rank RCCL path runs for real — bootstrap, collectives, graph capture — at
// loopback-socket speed: a correctness configuration, not a performance one.
bool ranks_share_devices();
// Device of a process-per-rank rank: LOCAL_RANK, modulo the visible devices when shared.
int rank_device(int local_rank);
// Sets the RCCL environment above for `rank` (rank < 0: only what bootstrap reads).
void prepare_shared_device_rccl(int rank);

class RcclComm final : public Comm {
 public:
  // 128-byte RCCL unique id (raw bytes), created by rank 0 and shared out of band.
  static std::string unique_id();
  // One process per GPU.
  RcclComm(const std::string& id, int rank, int world, int device);
  // One process, all listed devices (rank i <-> devices[i]).
  static std::vector<std::unique_ptr<Comm>> init_all(const std::vector<int>& devices);
  ~RcclComm() override;

  const char* kind() const override { return "rccl"; }
  int transport_world() const override;
  void allreduce_sum(const double* send, double* recv, size_t count, hipStream_t s) const override;
  void allgather(const double* send, double* recv, size_t count_per_rank,
                 hipStream_t s) const override;
  void broadcast(double* buf, size_t count, int root, hipStream_t s) const override;
  void reduce_sum(const double* send, double* recv, size_t count, int root,
                  hipStream_t s) const override;
  void check_async() const override;
  void abort() const override;
  // Thread-local capture: RCCL's own threads (proxy, bootstrap) may make HIP calls while a
  // rank's stream is capturing; in global mode any such call invalidates the capture, in
  // thread-local mode only this thread's calls are checked.
  void capture(Graph& g, hipStream_t s,
               const std::function<void(hipStream_t)>& body) const override {
    g.capture(s, body, hipStreamCaptureModeThreadLocal);
  }

  static void group_start();
  static void group_end();
  static std::string version();

 private:
  RcclComm(ncclComm_t c, int rank, int world, int device)
      : Comm(rank, world, device), comm_(c) {}
  mutable ncclComm_t comm_ = nullptr;  // nulled by abort()
};

// ------------------------------------------------------------------ loopback transport
constexpr int kMaxLoopbackRanks = 16;

class LoopbackGroup;

class LoopbackComm final : public Comm {
 public:
  LoopbackComm(LoopbackGroup* g, int rank);
  const char* kind() const override { return "loopback"; }
  int transport_world() const override { return world_; }
  void allreduce_sum(const double* send, double* recv, size_t count, hipStream_t s) const override;
  void allgather(const double* send, double* recv, size_t count_per_rank,
                 hipStream_t s) const override;
  void broadcast(double* buf, size_t count, int root, hipStream_t s) const override;
  void reduce_sum(const double* send, double* recv, size_t count, int root,
                  hipStream_t s) const override;
  void check_async() const override;
  void abort() const override;
  void capture(Graph& g, hipStream_t s,
               const std::function<void(hipStream_t)>& body) const override;
  void launch(const Graph& g, hipStream_t s) const override;
  bool capture_single_stream() const override { return true; }
  LoopbackGroup& group() const { return *g_; }

 private:
  LoopbackGroup* g_;  // the group owns its comms
};

// Shared state of W logical ranks on one device. Create it, hand comm(r) to the thread
// driving rank r (run_loopback does both).
class LoopbackGroup {
 public:
  static std::shared_ptr<LoopbackGroup> create(int world, int device, double timeout_s = 120.0);
  ~LoopbackGroup();
  int world() const { return world_; }
  int device() const { return device_; }
  const Comm* comm(int rank) const { return comms_.at(rank).get(); }
  // Host barrier over the W rank threads; throws after timeout_s or once the group is
  // broken (a rank failed: the others must not wait for it forever).
  void barrier(int rank);
  void mark_broken(const std::string& why);
  bool broken() const;
  // Collectives issued so far (rank 0's count) and group graph launches.
  long collectives() const { return collectives_; }
  long graph_launches() const { return graph_launches_; }

 private:
  friend class LoopbackComm;
  LoopbackGroup(int world, int device, double timeout_s);
  double* staging(int rank, size_t count, hipStream_t s);
  // s is the open group capture's stream: stream order replaces the event choreography
  bool shared(hipStream_t s) const { return capture_stream_ != nullptr && s == capture_stream_; }

  int world_, device_;
  double timeout_s_;
  std::vector<std::unique_ptr<Comm>> comms_;
  // barrier
  mutable std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  long generation_ = 0;
  bool broken_ = false;
  std::string why_;
  // Group captures: HIP's stream capture is not safe against several threads adding nodes
  // to one capture graph at once (heap corruption in launch-under-capture), so a rank holds
  // capture_mu_ for every HIP call it makes inside a group capture and drops it only while
  // it waits at a barrier.
  std::mutex capture_mu_;
  // collective state: pointers posted by each rank before the first barrier
  std::vector<const double*> send_;
  std::vector<double*> recv_;
  std::vector<std::unique_ptr<Event>> ready_, done_, pre_;
  Event post_;
  std::unique_ptr<Stream> origin_;
  std::vector<DeviceBuffer<double>> staging_;
  std::shared_ptr<Graph> captured_;  // rank 0's group capture, handed to every rank
  hipStream_t capture_stream_ = nullptr;  // origin_ while a group capture is open
  long collectives_ = 0, graph_launches_ = 0;
};

// Drive W logical ranks on `device`: one thread per rank runs fn(rank, comm). The first
// failure breaks the group (so no rank waits on a dead peer) and is rethrown.
void run_loopback(int world, int device, const std::function<void(int, const Comm*)>& fn,
                  double timeout_s = 120.0);

// ------------------------------------------------------------------ rank agreement
// Host values agreed over a communicator's ranks — what a multi-rank tool reports (the
// reference's clock stops on rank 0 only after every worker's MPI_Recv, riemann.cpp:82-93, so
// its time always covers the slowest worker):
//   barrier()  every rank's clock starts after it returns (a 1-double all-reduce, drained)
//   max(v)     the slowest rank's time        any(b)   a failure on one rank is every rank's
// A null comm is one rank (everything is the identity). Collective: every rank of the
// communicator calls the same methods in the same order. Each wait has the collective
// watchdog (a rank that never arrives aborts the communicator and throws instead of hanging).
class RankAgree {
 public:
  static constexpr size_t kMaxValues = 16;  // per rank per gather
  explicit RankAgree(const Comm* comm, double timeout_s = 300.0);
  ~RankAgree();
  RankAgree(const RankAgree&) = delete;
  RankAgree& operator=(const RankAgree&) = delete;
  int world() const { return comm_ ? comm_->world() : 1; }
  void barrier() const;
  // world x v.size() values in rank order (v.size() <= kMaxValues)
  std::vector<double> gather(const std::vector<double>& v) const;
  double max(double v) const;
  double min(double v) const;
  bool any(bool v) const;

 private:
  const Comm* comm_;
  double timeout_s_;
  hipStream_t s_ = nullptr;
  double* send_ = nullptr;  // device: kMaxValues
  double* recv_ = nullptr;  // device: world x kMaxValues
  double* host_ = nullptr;  // pinned: world x kMaxValues
};

// ------------------------------------------------------------------ RCCL transport evidence
// Which transport RCCL picked between the ranks. RCCL reports it only in its INIT log ("...
// via P2P/IPC", "... via NET/Socket/0", "nRanks 8 nNodes 1 localRanks 8"); a silent fallback
// off xGMI (P2P disabled, a leaked NCCL_HOSTID splitting one node into W "hosts") would
// otherwise go unrecorded. capture_rccl_log() routes RCCL's INIT-subsystem INFO lines into a
// per-process file (NCCL_DEBUG_FILE; not stdout) — it must run before the process's first
// RCCL call (RcclComm's constructors and unique_id() call it; MIINT_RCCL_LOG=0 turns it off)
// — and rccl_transport() parses what RCCL wrote so far. Peer connections are made at a
// communicator's first collective, so read it after one.
struct RcclTransport {
  std::string transport;   // distinct transports in first-seen order, '+'-joined: "P2P/IPC",
                           // "NET/Socket", "SHM/direct", ...; "" = no connection line seen
  int nranks = 0, nnodes = 0, local_ranks = 0;  // from "nRanks W nNodes N localRanks L"
  int connections = 0;     // "via" lines
  int comms = 0;           // "Init COMPLETE" lines
  std::string log;         // the file parsed ("" when RCCL logging is not captured)
  bool uses_net() const { return transport.find("NET/") != std::string::npos; }
};
RcclTransport parse_rccl_log(const std::string& text);
// "" or why a multi-rank record cannot stand (bench.py's transport_check, same rules): ranks
// of ONE node on distinct GPUs must be seen meeting over P2P (xGMI). Fail-closed: a network
// transport, more than one node counted, or no connection evidence at all is an error. Ranks
// sharing a GPU (share), one rank, and multi-node jobs (local_world != world) are exempt.
std::string transport_error(const RcclTransport& t, int world, int local_world, bool share);
// A user's own NCCL_DEBUG_FILE is honoured (read, never overwritten or deleted; "%h"/"%p"
// expanded as RCCL does); a user's own NCCL_DEBUG level below INFO still gets the INIT lines
// captured, and the WARN lines are echoed to stderr at exit (the user asked to see them).
void capture_rccl_log();
std::string rccl_log_path();  // "" when not capturing
RcclTransport rccl_transport();

// Minimal TCP rendezvous for native multi-process launches (no MPI in the image, and the
// CLI must not depend on Python): rank 0 listens on addr:port and hands the RCCL unique id
// to every other rank. Used when the CLI is launched by torchrun --no-python.
std::string rendezvous_unique_id(const std::string& addr, int port, int rank, int world,
                                 double timeout_s = 120.0);
// The transport underneath: rank 0 serves `payload` (exactly len bytes) to world - 1
// connections and returns it; every other rank connects (retrying until rank 0 listens)
// and returns the len bytes it received. Both sides fail after timeout_s.
std::string rendezvous_share(const std::string& addr, int port, int rank, int world,
                             const std::string& payload, size_t len, double timeout_s);

// Loopback kernels (loopback.hip): out[i] = sum over q < w of src[q][i], q in rank order.
struct LoopbackPtrs {
  const double* p[kMaxLoopbackRanks];
};
void launch_loopback_sum(const LoopbackPtrs& src, int w, size_t count, double* out,
                         hipStream_t s);

}  // namespace miint
