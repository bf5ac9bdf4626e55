// Native HIP runtime layer: devices, streams, events, buffers, graphs.
//
// Replaces the reference's host driver plumbing (cintegrate.cu:101-150):
//   * allocation happens once, outside anything timed or captured (H1);
//   * only the bytes that matter move, on pinned memory with hipMemcpyAsync (H2/H4:
//     the reference copies 288 MB of garbage over PCIe inside its timed region, B7);
//   * the integration step is captured once into a hipGraph and replayed (H3);
//   * every call is checked (B8).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstddef>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <utility>

#include "miint/common.hpp"

namespace miint {

struct DeviceInfo {
  int index = 0;
  std::string name;
  std::string arch;        // gcnArchName, e.g. "gfx950:sramecc+:xnack-"
  int num_cus = 0;         // multiProcessorCount (256 on MI355X)
  int clock_khz = 0;
  size_t total_mem = 0;
  int l2_bytes = 0;
  int max_threads_per_cu = 0;
  size_t lds_per_cu = 0;     // maxSharedMemoryPerMultiProcessor (160 KB on MI355X)
  size_t lds_per_block = 0;  // sharedMemPerBlock
};

int device_count();
DeviceInfo device_info(int device);
void set_device(int device);
int current_device();

// RAII device scope guard.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device);
  ~DeviceGuard();
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_;
};

class Stream {
 public:
  Stream();  // non-blocking stream on the current device
  explicit Stream(hipStream_t borrowed) : s_(borrowed), owned_(false) {}
  ~Stream();
  Stream(Stream&& o) noexcept : s_(o.s_), owned_(o.owned_) { o.s_ = nullptr; o.owned_ = false; }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  hipStream_t get() const { return s_; }
  void sync() const;

 private:
  hipStream_t s_ = nullptr;
  bool owned_ = true;
};

class Event {
 public:
  explicit Event(bool timing = true);
  ~Event();
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  void record(hipStream_t s);
  void sync() const;
  hipEvent_t get() const { return e_; }
  // Milliseconds between two recorded events.
  static float elapsed_ms(const Event& a, const Event& b);

 private:
  hipEvent_t e_ = nullptr;
};

template <typename T>
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t n) : n_(n) {
    if (n) MIINT_HIP(hipMalloc(&p_, n * sizeof(T)));
  }
  ~DeviceBuffer() { if (p_) (void)hipFree(p_); }
  DeviceBuffer(DeviceBuffer&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    return *this;
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  T* get() const { return p_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

// Page-locked host memory (hipHostMalloc) for async D2H/H2D. Allocated mapped + coherent
// (fine-grained), so kernels can also store results straight into it (device_ptr()):
// a finished kernel's stores are visible to the host after the stream synchronises.
template <typename T>
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t n) : n_(n) {
    if (n) {
      MIINT_HIP(hipHostMalloc(reinterpret_cast<void**>(&p_), n * sizeof(T),
                              hipHostMallocMapped | hipHostMallocPortable |
                                  hipHostMallocCoherent));
      std::memset(static_cast<void*>(p_), 0, n * sizeof(T));
      MIINT_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_), p_, 0));
    }
  }
  T* device_ptr() const { return d_; }
  ~PinnedBuffer() { if (p_) (void)hipHostFree(p_); }
  PinnedBuffer(PinnedBuffer&& o) noexcept : p_(o.p_), d_(o.d_), n_(o.n_) {
    o.p_ = nullptr;
    o.d_ = nullptr;
    o.n_ = 0;
  }
  PinnedBuffer& operator=(PinnedBuffer&& o) noexcept {
    std::swap(p_, o.p_);
    std::swap(d_, o.d_);
    std::swap(n_, o.n_);
    return *this;
  }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  T* get() const { return p_; }
  T& operator[](size_t i) const { return p_[i]; }
  size_t size() const { return n_; }

 private:
  T* p_ = nullptr;
  T* d_ = nullptr;
  size_t n_ = 0;
};

// Captured work on one stream, instantiated once and replayed.
//
// A Graph can also *adopt* a graph that a communicator captured for a whole group of
// ranks (LoopbackComm: one graph holds every logical rank's batch); such a graph is
// replayed through that communicator (launch_with), never directly.
class Graph {
 public:
  Graph() = default;
  ~Graph();
  Graph(const Graph&) = delete;
  Graph& operator=(const Graph&) = delete;
  // Capture everything `body` enqueues on `s` (global capture mode: any illegal
  // synchronising call inside body fails loudly instead of silently breaking capture).
  // Relaxed mode lets other threads enqueue onto streams that joined the capture
  // (group-wide captures).
  void capture(hipStream_t s, const std::function<void(hipStream_t)>& body,
               hipStreamCaptureMode mode = hipStreamCaptureModeGlobal);
  // Start / finish a capture whose body is enqueued by the caller (possibly from several
  // threads onto streams that joined `s`'s capture sequence).
  void begin(hipStream_t s, hipStreamCaptureMode mode);
  void end(hipStream_t s);
  void launch(hipStream_t s) const;
  void adopt(std::shared_ptr<const Graph> group) { reset(); group_ = std::move(group); }
  const Graph* group() const { return group_.get(); }
  bool ready() const { return exec_ != nullptr || group_ != nullptr; }
  size_t num_nodes() const { return group_ ? group_->num_nodes() : nodes_; }
  hipGraphExec_t exec() const { return exec_; }

 private:
  void reset();
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  size_t nodes_ = 0;
  std::shared_ptr<const Graph> group_;
};

// Monotonic wall clock in seconds (the reference's clock_gettime(CLOCK_MONOTONIC)).
inline double wall_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

// Process-start timestamp, captured by a static initialiser: the reference starts its
// clock before MPI_Init / context creation (riemann.cpp:51, cintegrate.cu:104), and the
// "%lf seconds" parity line reports from here.
double process_start_seconds();

}  // namespace miint
