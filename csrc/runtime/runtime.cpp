// Native HIP runtime layer implementation (see miint/runtime.hpp).
#include "miint/runtime.hpp"

#include "miint/kernels.hpp"

namespace miint {

namespace {
const double g_process_start = wall_seconds();
}  // namespace

double process_start_seconds() { return g_process_start; }

int device_count() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) return 0;
  MIINT_HIP(e);
  return n;
}

DeviceInfo device_info(int device) {
  hipDeviceProp_t prop;
  MIINT_HIP(hipGetDeviceProperties(&prop, device));
  DeviceInfo d;
  d.index = device;
  d.name = prop.name;
  d.arch = prop.gcnArchName;
  d.num_cus = prop.multiProcessorCount;
  d.clock_khz = prop.clockRate;
  d.total_mem = prop.totalGlobalMem;
  d.l2_bytes = prop.l2CacheSize;
  d.max_threads_per_cu = prop.maxThreadsPerMultiProcessor;
  d.lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
  d.lds_per_block = prop.sharedMemPerBlock;
  return d;
}

void fill_unset_slots(double* p, size_t count, hipStream_t stream) {
  if (count == 0) return;
  MIINT_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p),
                              static_cast<int>(kUnsetSlotWord), 2 * count, stream));
}

void set_device(int device) { MIINT_HIP(hipSetDevice(device)); }

int current_device() {
  int d = 0;
  MIINT_HIP(hipGetDevice(&d));
  return d;
}

DeviceGuard::DeviceGuard(int device) : prev_(current_device()) {
  if (device != prev_) set_device(device);
}
DeviceGuard::~DeviceGuard() { (void)hipSetDevice(prev_); }

Stream::Stream() { MIINT_HIP(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking)); }
Stream::~Stream() {
  if (owned_ && s_) (void)hipStreamDestroy(s_);
}
void Stream::sync() const { MIINT_HIP(hipStreamSynchronize(s_)); }

Event::Event(bool timing) {
  MIINT_HIP(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
}
Event::~Event() {
  if (e_) (void)hipEventDestroy(e_);
}
void Event::record(hipStream_t s) { MIINT_HIP(hipEventRecord(e_, s)); }
void Event::sync() const { MIINT_HIP(hipEventSynchronize(e_)); }
float Event::elapsed_ms(const Event& a, const Event& b) {
  float ms = 0.0f;
  MIINT_HIP(hipEventElapsedTime(&ms, a.e_, b.e_));
  return ms;
}

Graph::~Graph() { reset(); }

void Graph::reset() {
  if (exec_) { (void)hipGraphExecDestroy(exec_); exec_ = nullptr; }
  if (graph_) { (void)hipGraphDestroy(graph_); graph_ = nullptr; }
  nodes_ = 0;
  group_.reset();
}

void Graph::begin(hipStream_t s, hipStreamCaptureMode mode) {
  reset();
  MIINT_HIP(hipStreamBeginCapture(s, mode));
}

void Graph::end(hipStream_t s) {
  MIINT_HIP(hipStreamEndCapture(s, &graph_));
  MIINT_HIP(hipGraphGetNodes(graph_, nullptr, &nodes_));
  MIINT_HIP(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
}

void Graph::capture(hipStream_t s, const std::function<void(hipStream_t)>& body,
                    hipStreamCaptureMode mode) {
  begin(s, mode);
  try {
    body(s);
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
    throw;
  }
  end(s);
}

void Graph::launch(hipStream_t s) const {
  MIINT_CHECK(group_ == nullptr, "a group-captured graph is launched through its communicator");
  MIINT_CHECK(exec_ != nullptr, "graph not captured");
  MIINT_HIP(hipGraphLaunch(exec_, s));
}

}  // namespace miint
