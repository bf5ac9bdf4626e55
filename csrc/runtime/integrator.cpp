// RiemannPlan implementation (see miint/integrator.hpp).
#include "miint/integrator.hpp"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "miint/fault.hpp"
#include "miint/trace.hpp"

namespace miint {

namespace {
constexpr int kHostRing = 4096;  // pinned result slots for non-graph step loops
}

RiemannPlan::RiemannPlan(const RiemannConfig& cfg, int device, const Comm* comm)
    : cfg_(cfg), device_(device), comm_(comm), compute_((set_device(device), Stream())),
      comm_stream_(), ev_fork_(false), ev_join_(false) {
  MIINT_CHECK(cfg.n >= 1, "n must be >= 1");
  MIINT_CHECK(cfg.b != cfg.a, "empty interval");
  MIINT_CHECK(cfg.slots >= 1 && cfg.slots <= 64, "slots must be in [1, 64]");
  if (comm) {
    rank_ = comm->rank();
    world_ = comm->world();
    MIINT_CHECK(comm->device() == device, "communicator bound to another device");
  } else {
    MIINT_CHECK(cfg.world >= 1 && cfg.rank >= 0 && cfg.rank < cfg.world, "bad rank/world");
    rank_ = cfg.rank;
    world_ = cfg.world;
  }
  // Results go straight from the kernel into pinned host memory when nothing has to
  // happen to them on the device afterwards (no cross-GPU reduction by this plan).
  direct_ = cfg.host_direct && !(comm_ && (world_ > 1 || cfg.force_collective));
  DeviceGuard g(device);
  params_.a = cfg.a;
  params_.h = (cfg.b - cfg.a) / static_cast<double>(cfg.n);
  params_.off = rule_offset(cfg.rule);
  if (cfg.slice_world > 0) {
    MIINT_CHECK(cfg.slice_rank >= 0 && cfg.slice_rank < cfg.slice_world, "bad slice rank");
    rank_slice(cfg.n, cfg.slice_rank, cfg.slice_world, &params_.i_begin, &params_.n);
  } else {
    rank_slice(cfg.n, rank_, world_, &params_.i_begin, &params_.n);
  }
  params_.integrand = static_cast<int>(cfg.integrand);
  params_.ncoef = static_cast<int>(cfg.coef.size());
  MIINT_CHECK(cfg.coef.size() <= static_cast<size_t>(kMaxPolyCoeffs), "too many coefficients");
  for (size_t i = 0; i < cfg.coef.size(); ++i) params_.coef[i] = cfg.coef[i];
  params_.p0 = cfg.p0;
  params_.p1 = cfg.p1;
  scale_ = params_.h * integrand_scale(cfg.integrand);

  const DeviceInfo info = device_info(device);
  MIINT_CHECK(riemann_block_ok(cfg.block),
              "block must be 64, 128, 256, 512 or 1024 threads (got " + std::to_string(cfg.block) +
                  ")");
  const uint64_t bs = static_cast<uint64_t>(cfg.block);
  shape_ = default_riemann_shape(info.num_cus, cfg.waves_per_cu, cfg.block);
  if (cfg.grid > 0) shape_.grid = cfg.grid;
  // Never launch more workgroups than there are tiles to deal out, counted at the tile
  // length of the kernel that will run (32, 64 or 128 samples): idle workgroups still
  // launch, publish a partial and widen the final reduction.
  const uint64_t tl = static_cast<uint64_t>(riemann_tile_len(params_, cfg.dtype, cfg.div));
  const uint64_t tiles = (params_.n + tl - 1) / tl;
  const uint64_t need = std::max<uint64_t>(1, (tiles + bs - 1) / bs);
  shape_.grid = static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(shape_.grid), need));
  // Small N (latency-bound): give lanes ~4 tiles each, but keep >= 1 workgroup per CU. At
  // one tile per lane the launch, the partial stores and the final reduction over every
  // workgroup cost more than the extra rounds (table at 18e6 samples: 7.9 -> 6.4 us; pi4 at
  // 1e7: 6.0 -> 5.1 us; profiles/r1/small_n_grid.jsonl). N >= 2.7e8 keeps the full grid.
  // The grid is also rounded down to a whole number of workgroups per CU: at 275 workgroups
  // on 256 CUs, 19 CUs hold two and finish last (pi4 at 1e8: 17.9 us against 11.2 at 256).
  if (cfg.grid <= 0) {
    const uint64_t cus = static_cast<uint64_t>(info.num_cus);
    const uint64_t four =
        std::max<uint64_t>(cus, (tiles + 4 * bs - 1) / (4 * bs));
    uint64_t g = std::min<uint64_t>(static_cast<uint64_t>(shape_.grid), four);
    if (g > cus) g -= g % cus;
    shape_.grid = static_cast<int>(g);
  }
  // Multi-step batches keep every workgroup resident for a whole batch: the auto grid is
  // capped at the multi-step kernel's residency (pi4 fp64: 7 x 256-thread workgroups per CU,
  // 106 SGPRs); an explicit grid above it runs chained batches instead. The cap applies to
  // every path of such a plan (run(), direct steps, graphs), so all of them sum the same
  // partials, bit for bit. A plan whose batches can never run chained (unfused, or a
  // collective without bucketing) keeps the full grid and allocates no multi-step partials.
  MIINT_CHECK(cfg.close == "auto" || cfg.close == "kernel" || cfg.close == "launch",
              "close must be auto, kernel or launch (got " + cfg.close + ")");
  if (cfg.multistep && chained()) {
    // the in-launch close ("launch"; "auto" is the closing kernel) is its own instantiation,
    // with its own residency
    const int res_kernel =
        riemann_multistep_grid(params_, cfg.dtype, cfg.div, cfg.block, info.num_cus, false);
    close_launch_ = cfg.close == "launch";
    // 0: this integrand has no in-launch close (it closes with the kernel regardless)
    const int res_close =
        close_launch_
            ? riemann_multistep_grid(params_, cfg.dtype, cfg.div, cfg.block, info.num_cus, true)
            : 0;
    if (res_close == 0) close_launch_ = false;
    const int resident = close_launch_ ? res_close : res_kernel;
    if (resident > 0 && cfg.grid <= 0 && shape_.grid > resident) shape_.grid = resident;
    multistep_ = resident > 0 && shape_.grid <= resident;
    if (!multistep_) close_launch_ = false;
  }

  // chained batches: two partial halves per step stream
  const int lanes = step_streams(cfg.slots);
  partials_ = DeviceBuffer<double>(2 * static_cast<size_t>(std::max(1, lanes)) *
                                   static_cast<size_t>(shape_.grid));
  for (int l = 1; l < lanes; ++l) {
    step_streams_.emplace_back();
    ev_step_join_.emplace_back(new Event(false));
  }
  slots_ = DeviceBuffer<double>(static_cast<size_t>(shape_.grid));
  fill_unset_slots(slots_.get(), slots_.size(), nullptr);
  if (multistep_)
    ms_partials_ = DeviceBuffer<double>(static_cast<size_t>(cfg.slots) * shape_.grid);
  if (close_launch_) {
    ms_ticket_ = DeviceBuffer<unsigned int>(kTicketWords);
    MIINT_HIP(hipMemset(ms_ticket_.get(), 0, ms_ticket_.bytes()));
  }
  result_ = DeviceBuffer<double>(static_cast<size_t>(cfg.slots));
  sync_ = DeviceBuffer<double>(1);
  MIINT_HIP(hipMemset(sync_.get(), 0, sync_.bytes()));
  ticket_ = DeviceBuffer<unsigned int>(kTicketWords);
  MIINT_HIP(hipMemset(ticket_.get(), 0, ticket_.bytes()));
  MIINT_HIP(hipMemset(result_.get(), 0, result_.bytes()));
  if (cfg.integrand == Integrand::kTable) {
    MIINT_CHECK(cfg.table.size() >= 2, "table integrand needs a table");
    table_ = DeviceBuffer<double>(cfg.table.size());
    MIINT_HIP(hipMemcpy(table_.get(), cfg.table.data(), table_.bytes(), hipMemcpyHostToDevice));
  }
  host_ = PinnedBuffer<double>(static_cast<size_t>(std::max(kHostRing, cfg.slots)));
  for (int i = 0; i < cfg.slots; ++i) {
    ev_computed_.emplace_back(new Event(false));
    ev_drained_.emplace_back(new Event(false));
  }
  MIINT_HIP(hipDeviceSynchronize());
}

RiemannPlan::~RiemannPlan() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(compute_.get());
  (void)hipStreamSynchronize(comm_stream_.get());
  for (const auto& s : step_streams_) (void)hipStreamSynchronize(s.get());
}

DivMode RiemannPlan::effective_div() const {
  return miint::effective_div(cfg_.div, params_.h, cfg_.integrand, cfg_.dtype, params_.ncoef);
}

size_t RiemannPlan::graph_nodes() const {  // the largest captured batch graph
  size_t n = 0;
  for (const auto& kv : graphs_) n = std::max(n, kv.second->num_nodes());
  return n;
}

void RiemannPlan::enqueue_compute(hipStream_t s, int slot, int host_index) const {
  double* out = direct_ ? host_.device_ptr() + host_index : result_.get() + slot;
  const int tn = static_cast<int>(cfg_.table.size());
  if (cfg_.fused) {
    launch_riemann_fused(params_, cfg_.dtype, cfg_.div, shape_, table_.get(), tn,
                         slots_.get(), ticket_.get(), scale_, out, s);
  } else {
    launch_riemann_partials(params_, cfg_.dtype, cfg_.div, shape_, table_.get(), tn,
                            partials_.get(), s);
    launch_finalize(partials_.get(), shape_.grid, scale_, out, s, shape_.block);
  }
}

void RiemannPlan::enqueue_reduce(hipStream_t s, int slot) const {
  if (collective()) {  // without a native comm the caller reduces (torch path)
    double* v = result_.get() + slot;
    comm_->allreduce_sum(v, v, 1, s);
  }
}

void RiemannPlan::enqueue_copyout(hipStream_t s, int slot, int host_index) const {
  if (direct_) return;  // the kernel already stored into pinned memory
  MIINT_HIP(hipMemcpyAsync(host_.get() + host_index, result_.get() + slot, sizeof(double),
                           hipMemcpyDeviceToHost, s));
}

void RiemannPlan::enqueue(hipStream_t s, int slot, int host_index) const {
  enqueue_compute(s, slot, host_index);
  enqueue_reduce(s, slot);
  enqueue_copyout(s, slot, host_index);
}

double RiemannPlan::run() {
  DeviceGuard g(device_);
  enqueue(compute_.get(), 0, 0);
  compute_.sync();
  return host_[0];
}

// Steps j < nsteps use device slot j and host slot j. With overlap (and something to
// overlap), the reduce+copy chain runs on `rs` behind per-step events: a fork/join that
// hipStreamBeginCapture turns into graph edges.
// Chained batch: kernel j writes step j's partials into half j % 2 and finalizes step j-1
// from the other half into result slot j-1; a finalize kernel closes step nsteps-1.
void RiemannPlan::enqueue_chain(hipStream_t s, int nsteps) const {
  const int g = shape_.grid;
  const int tn = static_cast<int>(cfg_.table.size());
  for (int j = 0; j < nsteps; ++j) {
    double* cur = partials_.get() + static_cast<size_t>(j & 1) * g;
    const double* prev = j ? partials_.get() + static_cast<size_t>((j - 1) & 1) * g : nullptr;
    launch_riemann_chained(params_, cfg_.dtype, cfg_.div, shape_, table_.get(), tn, cur, prev, g,
                           scale_, j ? result_ptr(j - 1) : nullptr, s);
  }
  launch_finalize(partials_.get() + static_cast<size_t>((nsteps - 1) & 1) * g, g, scale_,
                  result_ptr(nsteps - 1), s, shape_.block);
}

int RiemannPlan::step_streams(int nsteps) const {
  if (!chained() || multistep_) return 1;
  const int want = cfg_.step_streams > 0            ? cfg_.step_streams
                   : params_.n >= kStepStreamsMaxCount ? 1
                                                       : kAutoStepStreams;
  return std::max(1, std::min(want, nsteps));
}

// Chained batch over L streams: step j runs on stream j % L (the compute stream is stream 0)
// as step j / L of that stream's own chain, with its own two partial halves; every chain
// closes with a finalize, and the compute stream joins all of them. The steps are
// independent integrations, so kernels on different streams may overlap (one's ramp and
// tail under another's work); each result is computed exactly as on one stream.
void RiemannPlan::enqueue_chain_streams(hipStream_t cs, int nsteps) {
  const int L = std::min(step_streams(nsteps), 1 + static_cast<int>(step_streams_.size()));
  if (L <= 1) {
    enqueue_chain(cs, nsteps);
    return;
  }
  const int g = shape_.grid;
  const int tn = static_cast<int>(cfg_.table.size());
  auto lane = [&](int l) { return l == 0 ? cs : step_streams_[static_cast<size_t>(l - 1)].get(); };
  auto half = [&](int l, int jj) {
    return partials_.get() + (2 * static_cast<size_t>(l) + static_cast<size_t>(jj & 1)) * g;
  };
  ev_fork_.record(cs);
  for (int l = 1; l < L; ++l) MIINT_HIP(hipStreamWaitEvent(lane(l), ev_fork_.get(), 0));
  for (int j = 0; j < nsteps; ++j) {
    const int l = j % L, jj = j / L;
    launch_riemann_chained(params_, cfg_.dtype, cfg_.div, shape_, table_.get(), tn, half(l, jj),
                           jj ? half(l, jj - 1) : nullptr, g, scale_,
                           jj ? result_ptr(j - L) : nullptr, lane(l));
  }
  for (int l = 0; l < L && l < nsteps; ++l) {
    const int last = l + ((nsteps - 1 - l) / L) * L;  // the chain's last step
    launch_finalize(half(l, last / L), g, scale_, result_ptr(last), lane(l), shape_.block);
    if (l > 0) {
      ev_step_join_[static_cast<size_t>(l - 1)]->record(lane(l));
      MIINT_HIP(hipStreamWaitEvent(cs, ev_step_join_[static_cast<size_t>(l - 1)]->get(), 0));
    }
  }
}

// A bucketed batch's step values (device slots 0 .. nsteps-1) -> every rank's global sums in
// pinned host slots 0 .. nsteps-1: the all-reduce writes them there itself
// (allreduce_to_host: RCCL's receive buffer is the mapped pinned memory), or it reduces in
// place and one copy follows.
void RiemannPlan::enqueue_bucket_reduce(hipStream_t s, int nsteps) const {
  const size_t n = static_cast<size_t>(nsteps);
  // (not inside a graph capture: RCCL may try to IPC-register a captured collective's
  // buffers, NCCL_GRAPH_REGISTER, which pinned host memory cannot be; the captured batch
  // keeps the device receive buffer and its copy node)
  if (allreduce_to_host() && !capturing_) {
    comm_->allreduce_sum(result_.get(), host_.device_ptr(), n, s);
    return;
  }
  comm_->allreduce_sum(result_.get(), result_.get(), n, s);
  MIINT_HIP(hipMemcpyAsync(host_.get(), result_.get(), sizeof(double) * n,
                           hipMemcpyDeviceToHost, s));
}

void RiemannPlan::check_allreduce_to_host() {
  if (ar_host_checked_ || !bucketed() || !cfg_.allreduce_to_host) return;
  ar_host_checked_ = true;
  DeviceGuard g(device_);
  hipStream_t s = compute_.get();
  const double want = 0.5 * static_cast<double>(world_) * (static_cast<double>(world_) + 1.0);
  const size_t probe = host_.size() - 1;  // the ring's last slot: rewritten before any use
  host_[probe] = std::numeric_limits<double>::quiet_NaN();
  host_[0] = static_cast<double>(rank_) + 1.0;
  MIINT_HIP(hipMemcpyAsync(result_.get(), host_.get(), sizeof(double), hipMemcpyHostToDevice, s));
  bool ok = true;
  try {
    comm_->allreduce_sum(result_.get(), host_.device_ptr() + probe, 1, s);
    if (cfg_.timeout_s > 0) wait_with_timeout(s, cfg_.timeout_s, comm_);
    else compute_.sync();
    ok = host_[probe] == want && !fault::allreduce_to_host_fails(rank_);
  } catch (const Error&) {
    ok = false;
    (void)hipGetLastError();
    compute_.sync();
  }
  // agree over the device-buffer path (sync_ is barrier()'s zero operand: restored)
  host_[0] = ok ? 0.0 : 1.0;
  MIINT_HIP(hipMemcpyAsync(sync_.get(), host_.get(), sizeof(double), hipMemcpyHostToDevice, s));
  comm_->allreduce_sum(sync_.get(), sync_.get(), 1, s);
  MIINT_HIP(hipMemcpyAsync(host_.get(), sync_.get(), sizeof(double), hipMemcpyDeviceToHost, s));
  MIINT_HIP(hipMemsetAsync(sync_.get(), 0, sizeof(double), s));
  if (cfg_.timeout_s > 0) wait_with_timeout(s, cfg_.timeout_s, comm_);
  else compute_.sync();
  ar_host_ok_ = host_[0] == 0.0;
}

void RiemannPlan::enqueue_batch(hipStream_t cs, hipStream_t rs, int nsteps, bool overlap) {
  if (chained()) {
    if (nsteps == 1)
      // a 1-step batch (a one-shot graph, a remainder): the fused launch, one kernel instead
      // of a 1-step persistent launch + its close kernel, or a chained launch + its finalize
      // (the same partials, the same order: bitwise the same value)
      launch_riemann_fused(params_, cfg_.dtype, cfg_.div, shape_, table_.get(),
                           static_cast<int>(cfg_.table.size()), slots_.get(), ticket_.get(),
                           scale_, result_ptr(0), cs);
    else if (multistep_)
      launch_riemann_multistep(params_, cfg_.dtype, cfg_.div, shape_, table_.get(),
                               static_cast<int>(cfg_.table.size()), ms_partials_.get(), nsteps,
                               scale_, result_ptr(0), cs,
                               close_launch_ ? ms_ticket_.get() : nullptr);
    else
      enqueue_chain_streams(cs, nsteps);
    if (bucketed()) {  // one all-reduce of all the batch's results
      enqueue_bucket_reduce(cs, nsteps);
      return;
    }
    // results in device slots (a single-GPU plan built with host_direct = false): one copy
    // of the batch's results into pinned memory
    if (!direct_)
      MIINT_HIP(hipMemcpyAsync(host_.get(), result_.get(), sizeof(double) * nsteps,
                               hipMemcpyDeviceToHost, cs));
    return;
  }
  if (bucketed()) {  // nsteps kernels, then one all-reduce of all their results
    for (int j = 0; j < nsteps; ++j) enqueue_compute(cs, j, j);
    enqueue_bucket_reduce(cs, nsteps);
    return;
  }
  if (!overlap || direct_ || !collective()) {
    for (int j = 0; j < nsteps; ++j) enqueue(cs, j, j);
    return;
  }
  ev_fork_.record(cs);
  MIINT_HIP(hipStreamWaitEvent(rs, ev_fork_.get(), 0));
  for (int j = 0; j < nsteps; ++j) {
    enqueue_compute(cs, j, j);
    ev_computed_[j]->record(cs);
    MIINT_HIP(hipStreamWaitEvent(rs, ev_computed_[j]->get(), 0));
    enqueue_reduce(rs, j);
    enqueue_copyout(rs, j, j);
  }
  ev_join_.record(rs);
  MIINT_HIP(hipStreamWaitEvent(cs, ev_join_.get(), 0));
}

void RiemannPlan::capture_graphs() { batch_graph(cfg_.slots); }

const Graph* RiemannPlan::batch_graph(int nsteps) {
  auto it = graphs_.find(nsteps);
  if (it != graphs_.end()) return it->second.get();
  if (!graph_error_.empty()) return nullptr;
  DeviceGuard g(device_);
  TraceRange tr("miint.plan.capture_graphs");
  if (collective() && graphs_.empty()) {
    // RCCL sets up peer connections lazily at a communicator's first collective: run that
    // one eagerly, outside the capture, so the graph only records steady-state operations.
    comm_->allreduce_sum(result_.get(), result_.get(), 1, compute_.get());
    MIINT_HIP(hipStreamSynchronize(compute_.get()));
  }
  std::unique_ptr<Graph> gr(new Graph());
  // A transport that captures a whole group on one stream gets the batch on that stream
  // only (no fork/join onto the comm stream).
  const bool one = collective() && comm_->capture_single_stream();
  try {
    capturing_ = true;
    capture_with(collective() ? comm_ : nullptr, *gr, compute_.get(), [&](hipStream_t s) {
      enqueue_batch(s, one ? s : comm_stream_.get(), nsteps, !one);
    });
    capturing_ = false;
  } catch (const Error& e) {
    capturing_ = false;
    // e.g. a collective that cannot be captured on this RCCL build: keep running with
    // direct stream enqueue (same results, more launch overhead) and say why.
    graph_error_ = e.what();
    (void)hipGetLastError();
    (void)hipStreamSynchronize(compute_.get());
    (void)hipStreamSynchronize(comm_stream_.get());
    if (collective() && std::string(comm_->kind()) == "loopback") throw;  // group is broken
    return nullptr;
  }
  return (graphs_[nsteps] = std::move(gr)).get();
}

void RiemannPlan::prepare_steps(int steps) {
  const int S = cfg_.slots;
  if (steps >= S) batch_graph(S);
  if (steps % S) batch_graph(steps % S);
}

// Capture (outside any timed region, if prepare_steps ran) the graphs `steps` replays.
bool RiemannPlan::use_graphs(bool requested, int steps) {
  if (!requested) return false;
  const int S = cfg_.slots;
  if (steps >= S && !batch_graph(S)) return false;
  if (steps % S && !batch_graph(steps % S)) return false;
  return true;
}

int RiemannPlan::host_index_of(int k, bool graphs) const {
  const bool batched = last_mode_ < 0 ? ((graphs && graphs_ready()) || bucketed() || multistep())
                                       : last_mode_ == 1;
  return batched ? k % cfg_.slots : k % host_capacity();
}

void RiemannPlan::launch_steps(int steps, bool pipeline, bool graphs) {
  DeviceGuard g(device_);
  TraceRange tr("miint.plan.launch_steps");
  check_allreduce_to_host();
  hipStream_t cs = compute_.get();
  hipStream_t rs = comm_stream_.get();
  const int S = cfg_.slots;
  const Comm* gc = collective() ? comm_ : nullptr;
  if (use_graphs(graphs, steps)) {
    last_mode_ = 1;
    if (steps >= S) {
      const Graph* full = batch_graph(S);
      for (int b = 0; b < steps / S; ++b) launch_with(gc, *full, cs);
      graph_launches_ += steps / S;
    }
    if (steps % S) {
      launch_with(gc, *batch_graph(steps % S), cs);
      ++graph_launches_;
    }
    return;
  }
  direct_steps_ += steps;
  last_mode_ = (bucketed() || multistep()) ? 1 : 0;
  if (bucketed() || multistep()) {  // whole batches enqueued directly (a multi-step batch is
                                    // two launches: no graph needed)
    for (int k = 0; k < steps; k += S) enqueue_batch(cs, rs, std::min(S, steps - k), false);
    return;
  }
  const bool overlap = pipeline && !direct_ && collective();
  for (int k = 0; k < steps; ++k) {
    const int slot = k % S;
    const int hidx = k % host_capacity();
    if (!overlap) {
      enqueue(cs, slot, hidx);
      continue;
    }
    if (k >= S) MIINT_HIP(hipStreamWaitEvent(cs, ev_drained_[slot]->get(), 0));
    enqueue_compute(cs, slot, hidx);
    ev_computed_[slot]->record(cs);
    MIINT_HIP(hipStreamWaitEvent(rs, ev_computed_[slot]->get(), 0));
    enqueue_reduce(rs, slot);
    enqueue_copyout(rs, slot, hidx);
    ev_drained_[slot]->record(rs);
  }
  if (overlap) {  // leave the compute stream ordered after the last copy
    ev_join_.record(rs);
    MIINT_HIP(hipStreamWaitEvent(cs, ev_join_.get(), 0));
  }
}

void RiemannPlan::sync() const {
  DeviceGuard g(device_);
  TraceRange tr("miint.plan.sync");
  if (collective() && cfg_.timeout_s > 0) {  // watchdog: a dead peer must not hang us forever
    wait_with_timeout(comm_stream_.get(), cfg_.timeout_s, comm_);
    wait_with_timeout(compute_.get(), cfg_.timeout_s, comm_);
    return;
  }
  compute_.sync();
  comm_stream_.sync();
}

void RiemannPlan::barrier() {
  if (!collective()) return;
  DeviceGuard g(device_);
  comm_->allreduce_sum(sync_.get(), sync_.get(), 1, compute_.get());
  if (cfg_.timeout_s > 0) wait_with_timeout(compute_.get(), cfg_.timeout_s, comm_);
  else compute_.sync();
}

StepTiming RiemannPlan::run_steps(int steps, bool pipeline, bool graphs) {
  DeviceGuard g(device_);
  check_allreduce_to_host();
  use_graphs(graphs, steps);
  StepTiming t;
  sync();
  barrier();  // no rank's clock starts before every rank is here
  const double w0 = wall_seconds();
  ev_t0_.record(compute_.get());
  launch_steps(steps, pipeline, graphs);
  fault::delay(rank_);            // MIINT_FAULT_*: a slow rank, for the agreement tests
  ev_t1_.record(compute_.get());  // every path leaves cs ordered after all of its work
  sync();
  t.wall_s = wall_seconds() - w0;
  t.device_ms = Event::elapsed_ms(ev_t0_, ev_t1_);
  t.steps = steps;
  return t;
}

BatchDiag RiemannPlan::diagnose_batch(int nsteps) {
  MIINT_CHECK(nsteps >= 1 && nsteps <= cfg_.slots, "diagnose_batch: 1 <= steps <= slots");
  DeviceGuard g(device_);
  TraceRange tr("miint.plan.diagnose_batch");
  check_allreduce_to_host();
  hipStream_t cs = compute_.get();
  const int tn = static_cast<int>(cfg_.table.size());
  BatchDiag d;
  d.steps = nsteps;
  // pass 1: the batch exactly as launch_steps enqueues it, between two events
  {
    Event a0, a1;
    sync();
    barrier();
    const double w0 = wall_seconds();
    a0.record(cs);
    enqueue_batch(cs, comm_stream_.get(), nsteps, false);
    a1.record(cs);
    sync();
    d.wall_us = (wall_seconds() - w0) * 1e6;
    d.device_us = Event::elapsed_ms(a0, a1) * 1e3;
  }
  // pass 2: the same operations with an event after every stage
  Event e0, e1, e2, e3, e4;
  sync();
  barrier();
  e0.record(cs);
  if (chained() && nsteps > 1 && multistep_) {
    launch_riemann_multistep(params_, cfg_.dtype, cfg_.div, shape_, table_.get(), tn,
                             ms_partials_.get(), nsteps, scale_, result_ptr(0), cs,
                             close_launch_ ? ms_ticket_.get() : nullptr, false);
    e1.record(cs);
    if (!close_launch_)
      launch_multistep_close(ms_partials_.get(), shape_.grid, nsteps, scale_, result_ptr(0),
                             shape_.block, cs);
  } else if (chained() && nsteps > 1) {
    enqueue_chain_streams(cs, nsteps);
    e1.record(cs);
  } else {  // fused launches, one per step (a 1-step batch, or an unchained plan)
    for (int j = 0; j < nsteps; ++j) enqueue_compute(cs, j, j);
    e1.record(cs);
  }
  e2.record(cs);
  if (bucketed()) {
    const size_t n = static_cast<size_t>(nsteps);
    if (allreduce_to_host()) {
      comm_->allreduce_sum(result_.get(), host_.device_ptr(), n, cs);
      e3.record(cs);
    } else {
      comm_->allreduce_sum(result_.get(), result_.get(), n, cs);
      e3.record(cs);
      MIINT_HIP(hipMemcpyAsync(host_.get(), result_.get(), sizeof(double) * n,
                               hipMemcpyDeviceToHost, cs));
    }
  } else {
    for (int j = 0; j < nsteps; ++j) enqueue_reduce(cs, j);
    e3.record(cs);
    for (int j = 0; j < nsteps; ++j) enqueue_copyout(cs, j, j);
  }
  e4.record(cs);
  sync();
  last_mode_ = 1;
  d.staged_us = Event::elapsed_ms(e0, e4) * 1e3;
  // one event's price: back-to-back events on the now idle stream
  {
    Event m[9];
    for (Event& e : m) e.record(cs);
    MIINT_HIP(hipStreamSynchronize(cs));
    std::vector<double> gaps;
    for (int i = 1; i < 9; ++i) gaps.push_back(Event::elapsed_ms(m[i - 1], m[i]) * 1e3);
    std::nth_element(gaps.begin(), gaps.begin() + 4, gaps.end());
    d.marker_us = gaps[4];
  }
  const double m = d.marker_us;
  d.compute_us = Event::elapsed_ms(e0, e1) * 1e3 - m;
  d.close_us = std::max(0.0, Event::elapsed_ms(e1, e2) * 1e3 - m);
  d.allreduce_us = std::max(0.0, Event::elapsed_ms(e2, e3) * 1e3 - m);
  d.copy_us = std::max(0.0, Event::elapsed_ms(e3, e4) * 1e3 - m);
  return d;
}

OneShotTiming RiemannPlan::time_one_shot(int reps, const std::string& mode, int warmup) {
  MIINT_CHECK(reps >= 1 && warmup >= 0, "time_one_shot: reps >= 1");
  MIINT_CHECK(!collective(), "time_one_shot: single-rank plans only");
  const bool graph = mode == "graph" || mode == "graph_poll";
  const bool poll = mode == "direct_poll" || mode == "graph_poll";
  MIINT_CHECK(graph || poll || mode == "direct",
              "time_one_shot mode: direct|direct_poll|graph|graph_poll");
  MIINT_CHECK(!poll || direct_, "a polled one-shot needs the result stored straight into pinned "
                                "memory (single GPU, host_direct)");
  DeviceGuard g(device_);
  hipStream_t cs = compute_.get();
  const Graph* g1 = graph ? batch_graph(1) : nullptr;
  MIINT_CHECK(!graph || g1, "time_one_shot: 1-step graph capture failed: " + graph_error_);
  // poll target: the host slot the launch stores into (step 0 of a batch, or run()'s slot 0)
  volatile uint64_t* word = reinterpret_cast<volatile uint64_t*>(host_.get());
  constexpr uint64_t kSentinel = 0x7ff8dead5eed0001ull;  // a NaN no integration produces
  std::vector<double> host_us, dev_us;
  double first = 0.0;
  // after the warm-up, calls alternate: host-timed ones without events (an event record is
  // an API call and a queue packet of its own: neither belongs in the interval), and
  // event-timed ones for the device span
  for (int i = 0; i < warmup + 2 * reps; ++i) {
    const bool events = i >= warmup && (i - warmup) % 2 == 1;
    MIINT_HIP(hipStreamSynchronize(cs));  // every call starts from an idle stream
    *word = kSentinel;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const double t0 = wall_seconds();
    if (events) ev_t0_.record(cs);
    if (graph) g1->launch(cs);
    else enqueue(cs, 0, 0);
    if (events) ev_t1_.record(cs);
    if (poll) {
      // bounded spin: past 50 ms (a healthy call takes ~80 us) the stream is
      // asked whether it finished or failed without storing the result; past the plan's
      // timeout (or 60 s) the call is abandoned
      const double limit = cfg_.timeout_s > 0 ? cfg_.timeout_s : 60.0;
      for (uint32_t spin = 1; *word == kSentinel; ++spin) {
        if ((spin & 1023u) != 0) continue;
        const double waited = wall_seconds() - t0;
        if (waited < 0.05) continue;
        const hipError_t q = hipStreamQuery(cs);
        if (q != hipErrorNotReady && *word == kSentinel) {
          MIINT_HIP(q);  // an asynchronous kernel failure surfaces here
          throw Error("time_one_shot: the stream finished but the result word was never stored");
        }
        if (waited > limit)
          throw Error("time_one_shot: no result after " + std::to_string(limit) + " s (" + mode + ")");
      }
    } else {
      MIINT_HIP(hipStreamSynchronize(cs));
    }
    const double t1 = wall_seconds();
    MIINT_HIP(hipStreamSynchronize(cs));
    uint64_t bits = *word;
    double v;
    std::memcpy(&v, &bits, sizeof(v));
    if (!direct_) v = host_[0];
    if (i == 0) first = v;
    MIINT_CHECK(std::memcmp(&v, &first, sizeof(v)) == 0,
                "time_one_shot: calls disagree (" + std::to_string(v) + " vs " +
                    std::to_string(first) + ")");
    if (i < warmup) continue;
    if (events) dev_us.push_back(static_cast<double>(Event::elapsed_ms(ev_t0_, ev_t1_)) * 1e3);
    else host_us.push_back((t1 - t0) * 1e6);
  }
  last_mode_ = graph ? 1 : 0;
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    const size_t n = v.size();
    return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
  };
  OneShotTiming r;
  r.mode = mode;
  r.reps = reps;
  r.median_us = med(host_us);
  r.min_us = *std::min_element(host_us.begin(), host_us.end());
  r.max_us = *std::max_element(host_us.begin(), host_us.end());
  r.device_median_us = med(dev_us);
  r.device_min_us = *std::min_element(dev_us.begin(), dev_us.end());
  r.value = first;
  return r;
}

}  // namespace miint
