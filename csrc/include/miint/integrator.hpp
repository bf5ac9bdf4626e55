// Integration plans: the user-facing native API.
//
// A RiemannPlan owns everything one rank needs to integrate f over [a, b] with n samples:
// its 64-bit slice of the sample range, the kernel launch shape, device workspace, a ring
// of result slots, pinned host results, and (optionally) an RCCL communicator for the
// cross-GPU sum. One integration ("step") is three stream-ordered stages:
//
//   compute  : fused Riemann kernel -> this rank's scaled partial (device slot, or, on a
//              single GPU, straight into mapped pinned host memory: no copy at all)
//   reduce   : RCCL allreduce of the slot across ranks over xGMI     [world > 1]
//   copyout  : 8-byte hipMemcpyAsync of the slot into pinned memory  [world > 1]
//
// Steps are replayed from hipGraphs that hold a whole batch of `slots` steps (one graph
// launch per batch). By default a batch is `slots` chained kernels (kernel k finalizes step
// k-1, no ticket) and one finalize kernel; on >1 GPU it then ends in ONE all-reduce of all
// its step results and one copy to pinned memory (bucketed). With bucket = false each step's
// all-reduce + copy runs on the comm stream (fork/join), overlapping the next kernel.
//
// Reference mapping: riemann.cpp:47-101 (MPI master/worker) and cintegrate.cu:101-150
// (CUDA host driver) are both instances of this plan (see csrc/cli/).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "miint/comm.hpp"
#include "miint/common.hpp"
#include "miint/kernels.hpp"
#include "miint/runtime.hpp"

namespace miint {

// Default number of concurrent step streams in a chained graph batch. One integration's
// kernel spends ~2-3 us ramping up, draining and flushing; with consecutive steps on
// different streams (independent: own partials, own result) the next step fills the CUs
// the previous one's tail leaves idle. 1/8 of N = 1e9 on one MI355X: 12.2 -> 11.2 us per
// step (20-step graphs), 11.5 -> 9.8-10.3 (48-step); 1/4: 20.5 -> 18.7; 1/2: 38.4 -> 36.8
// (profiles/r3/strong_slices_streams.jsonl, ss20.jsonl). A step that fills the whole GPU for
// ~70 us (>= kStepStreamsMaxCount samples: N = 1e9 on one GPU) gains nothing and replays
// less evenly (20-step graphs: 74.3 us on one stream, 74.2-88 on 2-4), so it keeps one.
constexpr int kAutoStepStreams = 4;
constexpr uint64_t kStepStreamsMaxCount = 600000000ull;

struct RiemannConfig {
  Integrand integrand = Integrand::kPi4;
  double a = 0.0, b = 1.0;
  uint64_t n = 1000000000ull;  // total samples over all ranks
  Rule rule = Rule::kLeft;
  DType dtype = DType::kF64;
  DivMode div = DivMode::kSeriesExact;  // exact-grade per point (common.hpp); --div series: the g-fold
  std::vector<double> coef;    // Integrand::kPoly
  double p0 = 0.0, p1 = 0.0;   // Integrand::kTrainVel (ts, vs)
  std::vector<double> table;   // Integrand::kTable (host copy, uploaded once)
  int grid = 0;                // workgroups; 0 = auto (waves_per_cu per CU)
  int block = kRiemannBlock;   // threads per workgroup: 64, 128, 256, 512 or 1024 (--block)
  int waves_per_cu = 32;       // 8 x 256-thread workgroups per CU (every Riemann kernel fits 8
                               // waves/SIMD): the default grid is one full wave
  bool fused = true;           // one launch (ticket reduction) vs partials + finalize
  bool chain = true;           // fused graph batches: kernel k finalizes step k-1 (no ticket;
                               // launch_riemann_chained), one finalize closes the batch
  bool host_direct = true;     // world == 1: kernel stores the result into pinned memory
  int slots = 16;              // steps per graph batch = result ring depth
  bool bucket = true;          // collective: ONE all-reduce of a batch's `slots` step results
                               // (every step still gets its own global sum) instead of one
                               // 8-byte all-reduce per step (~18 us each, not hidden: the
                               // kernels hold every CU slot the RCCL kernel would need)
  int rank = 0, world = 1;     // slice of [0, n) when no communicator is given (e.g. the
                               // torch.distributed path reduces results itself)
  bool force_collective = false;  // run the RCCL stage even with a 1-rank communicator
                                  // (exercises the multi-GPU graph path on one GPU)
  bool multistep = true;        // chained graph batches as ONE persistent launch of all the
                                // batch's steps plus one closing kernel
                                // (launch_riemann_multistep): one launch ramp and drain per
                                // batch instead of per step. The plan's grid is then capped at
                                // the multi-step kernel's residency (auto grid), so every path
                                // of the plan sums the same partials: values bit for bit equal.
                                // An explicit grid above residency turns it off.
  // How a multi-step batch is closed (its step partials summed into step values):
  //   "kernel": a closing kernel of one workgroup per step after the persistent launch;
  //   "launch": inside the persistent launch (handoff.hpp close_batch_in_launch): the last
  //             arrivals close it, no second kernel and no kernel boundary;
  //   "auto":   the closing kernel: the in-launch close measured equal at G = 1 and at every
  //             per-GPU share of an 8-GPU step (profiles/r6/batch_tail.md).
  // Both give the same values bit for bit. Kernels under the 8-wave hint close by the kernel
  // whatever is asked (the close code would spill there).
  std::string close = "auto";
  // Bucketed batches all-reduce their step values straight into the pinned host slots
  // (RCCL's receive buffer is the mapped host memory) instead of in place on the device
  // followed by a copy to pinned memory: one stream operation and one kernel boundary fewer.
  // Directly enqueued batches only: a captured batch graph keeps the device buffer + copy.
  bool allreduce_to_host = true;
  int step_streams = 0;         // chained graph batches: steps dealt round-robin to this many
                                // streams (each its own chain, ramp and tail of one step
                                // overlapping the next one's work); 0 = auto (kAutoStepStreams
                                // below kStepStreamsMaxCount samples per step, else 1)
  int slice_rank = 0, slice_world = 0;  // > 0: integrate rank slice_rank's share of [0, n) over
                                        // slice_world ranks whatever the communicator is (one-
                                        // GPU rehearsal of a strong-scaled run's per-GPU work)
  double timeout_s = 300.0;    // collective watchdog in sync(); <= 0 disables
};

// Balanced 64-bit slice of [0, n) for rank r of w: first (n % w) ranks get one extra.
inline void rank_slice(uint64_t n, int r, int w, uint64_t* begin, uint64_t* count) {
  const uint64_t q = n / static_cast<uint64_t>(w), rem = n % static_cast<uint64_t>(w);
  const uint64_t ur = static_cast<uint64_t>(r);
  *count = q + (ur < rem ? 1 : 0);
  *begin = ur * q + (ur < rem ? ur : rem);
}

struct StepTiming {
  double wall_s = 0.0;    // host wall clock around the whole run
  double device_ms = 0.0; // hipEvent time from first enqueue to last result
  int steps = 0;
};

// One integration per call, the reference's timing unit (cintegrate.cu:102-104,127-141 and
// riemann.cpp:49-51,90-93 clock exactly one run): host time from the launch call to the
// result readable in pinned host memory, and the device span of the same calls (hipEvents).
//   direct       one fused launch (last-workgroup ticket) + hipStreamSynchronize
//   direct_poll  the same launch; the host spins on the pinned result word the kernel
//                stores (single GPU, host_direct), no stream synchronisation in the interval
//   graph        a captured 1-step batch (+ its closing kernel) replayed + hipStreamSynchronize
//   graph_poll   the same replay, host spinning on the pinned result
// Every call starts from an idle stream; values are checked equal across calls. Host-timed
// calls record no events; the device span comes from as many event-timed calls in between.
struct OneShotTiming {
  std::string mode;
  int reps = 0;
  double median_us = 0.0, min_us = 0.0, max_us = 0.0;  // host: launch call -> result on host
  double device_median_us = 0.0, device_min_us = 0.0;  // hipEvent span of the same calls
  double value = 0.0;
};

// One batch of a plan taken apart by hipEvents between its stream stages (RiemannPlan::
// diagnose_batch; bench.py's untimed diagnostic batch on several GPUs). Microseconds.
// An event between two stages is a queue packet of its own whose release costs the device
// a few us (gfx950, ROCm 7.2: profiles/r6/batch_tail.md), so the batch runs twice: once between
// two events only (device_us, wall_us: the batch as the timed region runs it), once with an
// event after every stage (staged_us). marker_us is one event's own price, measured on the
// idle stream afterwards (the median gap between back-to-back events), and every stage below
// has it subtracted once. (Round 6 first priced an event as (staged_us - device_us) / 3: two
// runs of a 1.4 ms batch differ by more than three events, so at N = 1e9 that left ~4 us of
// event in every empty stage.) An event between two kernels also takes the place of the
// kernel boundary it sits in (the end-of-kernel release and the next dispatch), so the stages
// add up to less than the plain batch: boundary_us = device_us - compute_us - tail_us is that
// remainder (~5 us per batch on gfx950, plus the two passes' run-to-run spread).
struct BatchDiag {
  int steps = 0;
  double compute_us = 0.0;    // the batch's kernels up to the step values' partials (a multi-
                              // step launch with its in-launch close, or a chain)
  double close_us = 0.0;      // the closing kernel (~0: closed in the launch / by the chain)
  double allreduce_us = 0.0;  // the bucketed all-reduce (~0 without a collective)
  double copy_us = 0.0;       // the copy to pinned memory (~0: the all-reduce or the kernel
                              // stored there)
  double marker_us = 0.0;     // one event's own cost (see above)
  double device_us = 0.0;     // the batch between two events
  double staged_us = 0.0;     // the same batch with the stage events
  double wall_us = 0.0;       // host: launch call to every stage drained (the plan's sync)
  double tail_us() const { return close_us + allreduce_us + copy_us; }
  double boundary_us() const { return device_us - compute_us - tail_us(); }
};

class RiemannPlan {
 public:
  RiemannPlan(const RiemannConfig& cfg, int device, const Comm* comm = nullptr);
  ~RiemannPlan();
  RiemannPlan(const RiemannPlan&) = delete;
  RiemannPlan& operator=(const RiemannPlan&) = delete;

  const RiemannConfig& config() const { return cfg_; }
  int device() const { return device_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  uint64_t begin() const { return params_.i_begin; }
  uint64_t count() const { return params_.n; }
  double h() const { return params_.h; }
  double scale() const { return scale_; }
  LaunchShape shape() const { return shape_; }
  DivMode effective_div() const;
  bool direct() const { return direct_; }

  // Stage launchers. `slot` selects the device result slot, `host_index` the pinned slot.
  void enqueue_compute(hipStream_t s, int slot, int host_index) const;
  void enqueue_reduce(hipStream_t s, int slot) const;
  void enqueue_copyout(hipStream_t s, int slot, int host_index) const;
  void enqueue(hipStream_t s, int slot, int host_index) const;

  double* device_result(int slot) const { return result_.get() + slot; }
  double host_result(int host_index) const { return host_[host_index]; }
  int host_capacity() const { return static_cast<int>(host_.size()); }
  int slots() const { return cfg_.slots; }

  // One synchronous integration on the plan's own stream; returns the global value.
  double run();
  // Capture one batch of `slots` steps into a hipGraph (fork/join over two streams when
  // world > 1). Done lazily by the step runners.
  void capture_graphs();
  // Capture every graph launch_steps(steps, ., true) will replay: the `slots`-step batch
  // and, when slots does not divide steps, a batch of the remainder (so a timed run of any
  // length replays graphs only, and no capture lands inside it). Collective over ranks.
  void prepare_steps(int steps);
  // A batch graph has been captured (and no capture failed).
  bool graphs_ready() const { return !graphs_.empty() && graph_error_.empty(); }
  // Non-empty if graph capture failed (the plan then enqueues directly).
  const std::string& graph_error() const { return graph_error_; }
  size_t graph_nodes() const;
  // hipGraph replays issued so far (every launch_steps / run_steps call).
  long graph_launches() const { return graph_launches_; }
  // Steps enqueued directly (not from a graph) so far.
  long direct_steps() const { return direct_steps_; }

  // Run `steps` complete integrations back to back. graphs=true: whole batches of `slots`
  // steps as graph replays, then one replay of a remainder-sized batch graph (results of
  // step k in host slot k % slots).
  // graphs=false: direct enqueue (result of step k in host slot k % host_capacity); with
  // pipeline=true and world > 1 the reduce/copy of step k overlaps compute of step k+1.
  // bucketed(): batches of `slots` steps, one all-reduce each, host slot k % slots.
  // With a collective, every rank's clock starts after a collective barrier (barrier()).
  StepTiming run_steps(int steps, bool pipeline, bool graphs);
  // One batch of `nsteps` (<= slots) steps enqueued directly with hipEvents between its
  // stages (BatchDiag); the same operations and values as a timed batch, which it must not
  // be part of: the events are queue packets of their own. Collective over ranks (a barrier
  // first, and the batch's all-reduce). Results land in host slots 0 .. nsteps-1.
  BatchDiag diagnose_batch(int nsteps);
  // Collective: returns once every rank of the plan's communicator has entered (a 1-double
  // all-reduce, drained under the watchdog). No-op without a collective.
  void barrier();
  // See OneShotTiming. Single rank only. The warm-up calls are timed the same way and
  // dropped: from idle the clocks need a few hundred one-shot calls to settle (the fused
  // kernel runs 90 us on the first call and 75.5 us from about the 250th,
  // profiles/r4/oneshot_trace.md).
  OneShotTiming time_one_shot(int reps, const std::string& mode, int warmup = 400);
  // The same without synchronisation (bench.py brackets it with its own barrier + device
  // synchronize); call sync() before reading host results.
  void launch_steps(int steps, bool pipeline, bool graphs);
  void sync() const;
  // Host slot holding the result of step k of the last launch_steps/run_steps call (the
  // slot follows how that call actually ran: graph replays and bucketed batches use slot
  // k % slots, direct per-step enqueue k % host_capacity; `graphs` is only a fallback
  // before any call).
  int host_index_of(int k, bool graphs) const;
  hipStream_t compute_stream() const { return compute_.get(); }
  hipStream_t comm_stream() const { return comm_stream_.get(); }

  // True when this plan runs an RCCL reduction of its step results.
  bool collective() const { return comm_ && (world_ > 1 || cfg_.force_collective); }
  bool bucketed() const { return collective() && cfg_.bucket; }
  // Graph batches run chained kernels (see RiemannConfig::chain): single GPU, or bucketed.
  bool chained() const { return cfg_.fused && cfg_.chain && (!collective() || bucketed()); }
  // Chained batches run as one multi-step launch (RiemannConfig::multistep, in effect).
  bool multistep() const { return chained() && multistep_; }
  // Multi-step batches are closed inside the persistent launch (RiemannConfig::close).
  bool close_in_launch() const { return multistep() && close_launch_; }
  // Bucketed batches enqueued directly all-reduce into pinned host memory
  // (RiemannConfig::allreduce_to_host); captured batch graphs keep the device buffer + copy.
  // Off after check_allreduce_to_host found the transport unable to (every rank agrees).
  bool allreduce_to_host() const {
    return bucketed() && cfg_.allreduce_to_host && ar_host_ok_;
  }
  // Collective, once per plan before its first batch (launch_steps, run_steps,
  // diagnose_batch call it): one 1-double all-reduce of rank + 1 into pinned memory, checked
  // on the host against world (world + 1) / 2; a wrong value or an error on any rank (agreed
  // by a device-buffer all-reduce) turns allreduce_to_host off for the plan, so a transport
  // that cannot write host memory costs a copy, not the run.
  void check_allreduce_to_host();

 private:
  void enqueue_batch(hipStream_t cs, hipStream_t rs, int nsteps, bool overlap);
  void enqueue_bucket_reduce(hipStream_t s, int nsteps) const;
  void enqueue_chain(hipStream_t s, int nsteps) const;
  void enqueue_chain_streams(hipStream_t cs, int nsteps);
 public:
  // Streams a chained batch of `nsteps` steps runs on (1 = the compute stream only).
  int step_streams(int nsteps) const;
 private:
  const Graph* batch_graph(int nsteps);  // captured lazily; null if capture failed
  bool use_graphs(bool requested, int steps);
  double* result_ptr(int j) const { return direct_ ? host_.device_ptr() + j : result_.get() + j; }

  RiemannConfig cfg_;
  int device_;
  const Comm* comm_;
  int rank_ = 0, world_ = 1;
  bool direct_ = false;
  RiemannParams params_{};
  double scale_ = 1.0;
  LaunchShape shape_{1, kRiemannBlock};
  DeviceBuffer<double> partials_;  // 2 x grid: chained batches alternate halves (+ 2-kernel)
  DeviceBuffer<double> slots_;     // grid write-once slots of the fused (ticket) kernel
  DeviceBuffer<double> ms_partials_;  // multistep: slots x grid partials
  bool multistep_ = false;
  bool close_launch_ = false;         // multistep batches closed in-launch
  bool capturing_ = false;            // batch_graph() is capturing (enqueue_bucket_reduce)
  bool ar_host_ok_ = true;            // check_allreduce_to_host's verdict
  bool ar_host_checked_ = false;
  DeviceBuffer<unsigned int> ms_ticket_;  // its arrival counters (close_batch_in_launch)
  DeviceBuffer<double> result_;
  DeviceBuffer<double> sync_;      // barrier(): the 1-double all-reduce's operand
  DeviceBuffer<unsigned int> ticket_;
  DeviceBuffer<double> table_;
  PinnedBuffer<double> host_;
  Stream compute_;
  Stream comm_stream_;
  std::vector<Stream> step_streams_;  // concurrent chains of a batch (step_streams() of them)
  std::vector<std::unique_ptr<Event>> ev_step_join_;
  std::vector<std::unique_ptr<Event>> ev_computed_, ev_drained_;
  Event ev_fork_, ev_join_;
  Event ev_t0_, ev_t1_;
  std::map<int, std::unique_ptr<Graph>> graphs_;  // batch graphs by step count
  std::string graph_error_;
  long graph_launches_ = 0, direct_steps_ = 0;
  int last_mode_ = -1;  // last launch_steps: -1 none, 0 direct per-step, 1 batches/graphs
};

}  // namespace miint
