// LoopbackComm / LoopbackGroup: W logical ranks on one device (see miint/comm.hpp).
//
// The test transport that lets every world > 1 code path of the plans run on the one-GPU
// pool: RCCL refuses two ranks on one device, so here the "network" is cross-stream events
// plus a fixed-order sum kernel (loopback.hip), and the rendezvous is a host barrier.
#include <algorithm>
#include <chrono>
#include <thread>

#include "miint/comm.hpp"

namespace miint {

// Event discipline (why no stream can wait on an event that is re-recorded under it): each
// collective is  post pointer + record ready[r]  | barrier 1 |  wait ready[q], work, record
// done[r]  | barrier 2 |  wait done[q], copy-out. A rank re-records ready[r] only after
// barrier 2 (every wait on ready happened before it) and done[r] only after the next
// barrier 1 (every wait on done happened before it). Group launches use pre and post the
// same way.
namespace {
constexpr size_t kStagingInit = 1 << 16;  // doubles per rank, grown outside captures

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  MIINT_HIP(hipStreamIsCapturing(s, &st));
  return st != hipStreamCaptureStatusNone;
}
void wait_on(hipStream_t s, const Event& e) { MIINT_HIP(hipStreamWaitEvent(s, e.get(), 0)); }
// The group-capture lock this thread holds (null outside a group capture body).
thread_local std::mutex* t_capture_lock = nullptr;

// Holds `mu` for the scope and marks it as this thread's capture lock.
class CaptureLock {
 public:
  explicit CaptureLock(std::mutex& mu) : mu_(mu) {
    mu_.lock();
    t_capture_lock = &mu_;
  }
  ~CaptureLock() {
    t_capture_lock = nullptr;
    mu_.unlock();
  }

 private:
  std::mutex& mu_;
};
}  // namespace

LoopbackGroup::LoopbackGroup(int world, int device, double timeout_s)
    : world_(world), device_(device), timeout_s_(timeout_s),
      post_((set_device(device), false)) {
  MIINT_CHECK(world >= 1 && world <= kMaxLoopbackRanks,
              "loopback world must be in [1, " + std::to_string(kMaxLoopbackRanks) + "]");
  DeviceGuard g(device);
  origin_.reset(new Stream());
  send_.assign(world, nullptr);
  recv_.assign(world, nullptr);
  for (int r = 0; r < world; ++r) {
    ready_.emplace_back(new Event(false));
    done_.emplace_back(new Event(false));
    pre_.emplace_back(new Event(false));
    staging_.emplace_back(kStagingInit);
  }
}

std::shared_ptr<LoopbackGroup> LoopbackGroup::create(int world, int device, double timeout_s) {
  std::shared_ptr<LoopbackGroup> g(new LoopbackGroup(world, device, timeout_s));
  for (int r = 0; r < world; ++r) g->comms_.emplace_back(new LoopbackComm(g.get(), r));
  return g;
}

LoopbackGroup::~LoopbackGroup() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();  // staging / events may still be in use by queued work
}

void LoopbackGroup::barrier(int rank) {
  // inside a group capture: let the other ranks issue their HIP calls while we wait
  std::mutex* held = t_capture_lock;
  if (held) held->unlock();
  struct Relock {
    std::mutex* m;
    ~Relock() {
      if (m) m->lock();
    }
  } relock{held};
  std::unique_lock<std::mutex> lk(mu_);
  if (broken_) fail("loopback group broken: " + why_, __FILE__, __LINE__);
  const long gen = generation_;
  if (++arrived_ == world_) {
    arrived_ = 0;
    ++generation_;
    cv_.notify_all();
    return;
  }
  const bool ok = cv_.wait_for(lk, std::chrono::duration<double>(timeout_s_),
                               [&] { return generation_ != gen || broken_; });
  if (broken_) fail("loopback group broken: " + why_, __FILE__, __LINE__);
  if (!ok) {
    broken_ = true;
    why_ = "rank " + std::to_string(rank) + " waited " + std::to_string(timeout_s_) +
           " s at a barrier (a rank skipped a collective or died)";
    cv_.notify_all();
    fail("loopback " + why_, __FILE__, __LINE__);
  }
}

void LoopbackGroup::mark_broken(const std::string& why) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!broken_) {
    broken_ = true;
    why_ = why;
  }
  cv_.notify_all();
}

bool LoopbackGroup::broken() const {
  std::lock_guard<std::mutex> lk(mu_);
  return broken_;
}

double* LoopbackGroup::staging(int rank, size_t count, hipStream_t s) {
  DeviceBuffer<double>& b = staging_[rank];
  if (count > b.size()) {
    MIINT_CHECK(!capturing(s), "loopback collective of " + std::to_string(count) +
                                   " doubles inside a graph capture exceeds the staging buffer (" +
                                   std::to_string(b.size()) + "); run it once outside first");
    MIINT_HIP(hipStreamSynchronize(s));  // the old buffer may still be read by queued work
    b = DeviceBuffer<double>(std::max(count, 2 * b.size()));
  }
  return b.get();
}

LoopbackComm::LoopbackComm(LoopbackGroup* g, int rank)
    : Comm(rank, g->world(), g->device()), g_(g) {}

void LoopbackComm::allreduce_sum(const double* send, double* recv, size_t count,
                                 hipStream_t s) const {
  LoopbackGroup& G = *g_;
  const int r = rank_, W = world_;
  const bool ev = !G.shared(s);
  double* st = G.staging(r, count, s);
  G.send_[r] = send;
  if (ev) G.ready_[r]->record(s);
  G.barrier(r);
  LoopbackPtrs p{};
  for (int q = 0; q < W; ++q) {
    p.p[q] = G.send_[q];
    if (ev && q != r) wait_on(s, *G.ready_[q]);
  }
  if (count) launch_loopback_sum(p, W, count, st, s);
  if (ev) G.done_[r]->record(s);
  if (r == 0) ++G.collectives_;
  G.barrier(r);
  for (int q = 0; q < W; ++q)
    if (ev && q != r) wait_on(s, *G.done_[q]);  // every rank has read every send buffer
  if (count)
    // (hipMemcpyDefault: recv may be mapped pinned host memory, RiemannConfig::allreduce_to_host)
    MIINT_HIP(hipMemcpyAsync(recv, st, count * sizeof(double), hipMemcpyDefault, s));
}

void LoopbackComm::reduce_sum(const double* send, double* recv, size_t count, int root,
                              hipStream_t s) const {
  LoopbackGroup& G = *g_;
  const int r = rank_, W = world_;
  MIINT_CHECK(root >= 0 && root < W, "reduce root out of range");
  const bool ev = !G.shared(s);
  double* st = r == root ? G.staging(r, count, s) : nullptr;
  G.send_[r] = send;
  if (ev) G.ready_[r]->record(s);
  G.barrier(r);
  if (r == root) {
    LoopbackPtrs p{};
    for (int q = 0; q < W; ++q) {
      p.p[q] = G.send_[q];
      if (ev && q != r) wait_on(s, *G.ready_[q]);
    }
    if (count) {
      launch_loopback_sum(p, W, count, st, s);
      MIINT_HIP(hipMemcpyAsync(recv, st, count * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
  }
  if (ev) G.done_[r]->record(s);
  if (r == 0) ++G.collectives_;
  G.barrier(r);
  if (ev && r != root) wait_on(s, *G.done_[root]);  // root has read our send buffer
}

void LoopbackComm::allgather(const double* send, double* recv, size_t count,
                             hipStream_t s) const {
  LoopbackGroup& G = *g_;
  const int r = rank_, W = world_;
  const bool ev = !G.shared(s);
  G.send_[r] = send;
  if (ev) G.ready_[r]->record(s);
  G.barrier(r);
  for (int q = 0; q < W; ++q) {
    double* dst = recv + static_cast<size_t>(q) * count;
    if (ev && q != r) wait_on(s, *G.ready_[q]);
    if (count && dst != G.send_[q])  // in place (send == recv + r*count): nothing to move
      MIINT_HIP(hipMemcpyAsync(dst, G.send_[q], count * sizeof(double),
                               hipMemcpyDeviceToDevice, s));
  }
  if (ev) G.done_[r]->record(s);
  if (r == 0) ++G.collectives_;
  G.barrier(r);
  for (int q = 0; q < W; ++q)
    if (ev && q != r) wait_on(s, *G.done_[q]);
}

void LoopbackComm::broadcast(double* buf, size_t count, int root, hipStream_t s) const {
  LoopbackGroup& G = *g_;
  const int r = rank_, W = world_;
  MIINT_CHECK(root >= 0 && root < W, "broadcast root out of range");
  const bool ev = !G.shared(s);
  G.send_[r] = buf;
  if (ev) G.ready_[r]->record(s);
  G.barrier(r);
  if (r != root) {
    if (ev) wait_on(s, *G.ready_[root]);
    if (count)
      MIINT_HIP(hipMemcpyAsync(buf, G.send_[root], count * sizeof(double),
                               hipMemcpyDeviceToDevice, s));
  }
  if (ev) G.done_[r]->record(s);
  if (r == 0) ++G.collectives_;
  G.barrier(r);
  if (ev && r == root)
    for (int q = 0; q < W; ++q)
      if (q != r) wait_on(s, *G.done_[q]);  // nobody still reads root's buffer
}

void LoopbackComm::check_async() const {
  if (g_->broken()) fail("loopback group broken", __FILE__, __LINE__);
}

void LoopbackComm::abort() const { g_->mark_broken("aborted by rank " + std::to_string(rank_)); }

// Group capture on ONE stream (origin_): rank 0 opens the capture, every rank enqueues its
// body onto origin_ holding capture_mu_ (released only inside barriers), rank 0 closes it.
// Within the body, stream order on origin_ plus the collectives' barriers give every
// dependency the event choreography gives the uncaptured path: all pre-collective work of
// every rank is enqueued before any rank's post-collective work.
void LoopbackComm::capture(Graph& g, hipStream_t /*s*/,
                           const std::function<void(hipStream_t)>& body) const {
  LoopbackGroup& G = *g_;
  const int r = rank_;
  G.barrier(r);
  if (r == 0) {
    G.captured_ = std::make_shared<Graph>();
    G.captured_->begin(G.origin_->get(), hipStreamCaptureModeRelaxed);
    G.capture_stream_ = G.origin_->get();
  }
  G.barrier(r);
  try {
    CaptureLock cl(G.capture_mu_);
    body(G.origin_->get());
  } catch (const std::exception& e) {
    G.mark_broken("rank " + std::to_string(r) + " failed inside a group capture: " + e.what());
    if (r == 0) {
      hipGraph_t dead = nullptr;
      (void)hipStreamEndCapture(G.origin_->get(), &dead);
      if (dead) (void)hipGraphDestroy(dead);
      G.capture_stream_ = nullptr;
    }
    throw;
  }
  G.barrier(r);
  if (r == 0) {
    G.capture_stream_ = nullptr;
    G.captured_->end(G.origin_->get());
  }
  G.barrier(r);
  g.adopt(G.captured_);
  G.barrier(r);  // every rank holds the graph before rank 0 may replace captured_
}

void LoopbackComm::launch(const Graph& g, hipStream_t s) const {
  LoopbackGroup& G = *g_;
  const int r = rank_;
  const Graph* shared = g.group();
  MIINT_CHECK(shared != nullptr, "loopback launch of a graph it did not capture");
  G.pre_[r]->record(s);
  G.barrier(r);
  if (r == 0) {
    hipStream_t o = G.origin_->get();
    for (int q = 0; q < world_; ++q) wait_on(o, *G.pre_[q]);
    MIINT_HIP(hipGraphLaunch(shared->exec(), o));
    G.post_.record(o);
    ++G.graph_launches_;
  }
  G.barrier(r);
  wait_on(s, G.post_);
}

void run_loopback(int world, int device, const std::function<void(int, const Comm*)>& fn,
                  double timeout_s) {
  std::shared_ptr<LoopbackGroup> grp = LoopbackGroup::create(world, device, timeout_s);
  std::vector<std::thread> th;
  std::mutex mu;
  std::string err;
  for (int r = 0; r < world; ++r) {
    th.emplace_back([&, r] {
      try {
        set_device(device);
        fn(r, grp->comm(r));
      } catch (const std::exception& e) {
        {
          std::lock_guard<std::mutex> g(mu);
          if (err.empty()) err = "rank " + std::to_string(r) + ": " + e.what();
        }
        grp->mark_broken(std::string("rank ") + std::to_string(r) + " failed: " + e.what());
      }
    });
  }
  for (auto& x : th) x.join();
  if (!err.empty()) throw Error(err);
}

}  // namespace miint
