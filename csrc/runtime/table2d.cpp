// Table2DPlan implementation (see miint/table2d.hpp).
#include "miint/table2d.hpp"

#include <algorithm>

#include "miint/fault.hpp"
#include "miint/integrator.hpp"
#include "miint/oracle.hpp"
#include "miint/trace.hpp"

namespace miint {

Table2DPlan::Table2DPlan(const Table2DConfig& cfg, int device, const Comm* comm)
    : cfg_(cfg), device_(device), comm_(comm), stream_((set_device(device), Stream())) {
  MIINT_CHECK(cfg.grid >= 1 && cfg.grid <= (1 << 20), "grid out of range");
  if (comm && comm->world() > 1) {
    rank_ = comm->rank();
    world_ = comm->world();
  } else {  // no communicator, or a 1-rank one (force_collective): the configured row slice
    MIINT_CHECK(cfg.world >= 1 && cfg.rank >= 0 && cfg.rank < cfg.world, "bad slice rank/world");
    rank_ = cfg.rank;
    world_ = cfg.world;
  }
  collective_ = comm && (comm->world() > 1 || cfg.force_collective);
  uint64_t b = 0, c = 0;
  rank_slice(static_cast<uint64_t>(cfg.grid), rank_, world_, &b, &c);
  row0_ = static_cast<int>(b);
  row1_ = static_cast<int>(b + c);
  const auto& prof = oracle::profile_table();
  const int n = static_cast<int>(prof.size());
  v_ = DeviceBuffer<double>(prof.size());
  table_ = DeviceBuffer<double>(static_cast<size_t>(n) * n);
  MIINT_HIP(hipMemcpy(v_.get(), prof.data(), v_.bytes(), hipMemcpyHostToDevice));
  launch_outer_product(v_.get(), n, table_.get(), stream_.get());
  // bucketed_ first: chained() (and so the multi-step choice and chain count) depends on it
  bucketed_ = cfg.bucket && collective_;
  const int cus = device_info(device).num_cus;
  const auto params = [&](int min_wg) {
    return Table2DParams{table_.get(), n, n, cfg.extent, cfg.extent, cfg.grid, cfg.grid,
                         row0_, std::max(row1_, row0_ + 1), min_wg};
  };
  // A multi-step plan takes the most rows per wave that fit (min_wg 1): its step phases give
  // the parallelism. Every launch of the plan (run(), the replay) uses that same shape, so
  // all its paths sum the same partials (bitwise equal).
  if (cfg.multistep && cfg.min_wg == 0 && chained() && row1_ > row0_ &&
      table2d_multistep_ok(params(1), cus))
    cfg_.min_wg = 1;
  const Table2DParams p = params(cfg_.min_wg);
  partials_ = DeviceBuffer<double>(static_cast<size_t>(table2d_grid(p)));
  multistep_ = cfg.multistep && row1_ > row0_ && table2d_multistep_ok(p, cus);
  resident_per_cu_ = table2d_multistep_resident(p);
  MIINT_CHECK(cfg.graph_steps >= 0 && cfg.graph_steps <= kT2MaxReplaySteps,
              "table2d: graph_steps 0 (auto) or 1..kT2MaxReplaySteps");
  if (cfg.graph_steps > 0) {
    graph_steps_ = cfg.graph_steps;
  } else if (cfg.multistep && chained()) {
    // from the configuration only: every rank of a collective plan must replay the same
    // count, its all-reduce covering graph_steps_ values
    graph_steps_ = table2d_auto_graph_steps(cfg.grid, cfg.extent, world_);
  }
  if (multistep_) {
    ms_partials_ = DeviceBuffer<double>(static_cast<size_t>(graph_steps_) * partials_.size());
    phases_ = std::max(1, table2d_multistep_phases(p, cus, graph_steps_, cfg.phases));
  }
  const int L = (!chained() || multistep_)
                    ? 1
                    : std::max(1, std::min(graph_steps_, cfg_.step_streams > 0 ? cfg_.step_streams
                                                                              : kAutoT2Streams));
  // chained launches: a double buffer per chain
  chain_ = DeviceBuffer<double>(2 * static_cast<size_t>(L) * partials_.size());
  for (int l = 1; l < L; ++l) {
    lanes_.emplace_back();
    ev_join_.emplace_back(new Event(false));
  }
  fill_unset_slots(partials_.get(), partials_.size(), stream_.get());  // fused kernel's slots
  result_ = DeviceBuffer<double>(static_cast<size_t>(graph_steps_));
  sync_ = DeviceBuffer<double>(1);
  MIINT_HIP(hipMemset(sync_.get(), 0, sync_.bytes()));
  ticket_ = DeviceBuffer<unsigned int>(kTicketWords);
  MIINT_HIP(hipMemset(ticket_.get(), 0, ticket_.bytes()));
  host_ = PinnedBuffer<double>(static_cast<size_t>(graph_steps_));
  stream_.sync();
}

// the chains a chained replay actually runs: the plan's stream plus its lane streams
int Table2DPlan::step_streams() const { return 1 + static_cast<int>(lanes_.size()); }

void Table2DPlan::barrier() {
  if (!collective_) return;
  comm_->allreduce_sum(sync_.get(), sync_.get(), 1, stream_.get());
  wait_with_timeout(stream_.get(), 300.0, comm_);
}

void Table2DPlan::launch_local(double* out, hipStream_t s) {
  const int n = static_cast<int>(oracle::profile_table().size());
  if (row1_ > row0_) {
    const Table2DParams p{table_.get(), n, n, cfg_.extent, cfg_.extent, cfg_.grid, cfg_.grid,
                          row0_, row1_, cfg_.min_wg};
    launch_table2d_fused(p, partials_.get(), ticket_.get(), out, s);
  } else {
    MIINT_HIP(hipMemsetAsync(out, 0, sizeof(double), s));  // more ranks than rows
  }
}

void Table2DPlan::enqueue(hipStream_t s) {
  const bool multi = collective_;
  // one rank: the kernel's last workgroup stores straight into mapped pinned memory
  launch_local(multi ? result_.get() : host_.device_ptr(), s);
  if (!multi) return;
  comm_->allreduce_sum(result_.get(), result_.get(), 1, s);
  MIINT_HIP(hipMemcpyAsync(host_.get(), result_.get(), sizeof(double), hipMemcpyDeviceToHost, s));
}

double Table2DPlan::run() {
  DeviceGuard g(device_);
  enqueue(stream_.get());
  stream_.sync();
  last_batched_ = false;
  return host_[0];
}

double Table2DPlan::time(int iters, bool graphs) {
  DeviceGuard g(device_);
  hipStream_t s = stream_.get();
  if (!graphs) {
    enqueue(s);  // warm
    stream_.sync();
    barrier();  // no rank's clock starts before every rank is here
    e0_.record(s);
    for (int i = 0; i < iters; ++i) enqueue(s);
    fault::delay(rank_);
    e1_.record(s);
    stream_.sync();
    return Event::elapsed_ms(e0_, e1_) / iters;
  }
  const Comm* gc = collective_ ? comm_ : nullptr;  // group-wide graphs (loopback)
  const bool multi = gc != nullptr;
  const bool batched = !multi || bucketed_;  // graph_steps_ results land in one replay
  if (!graph_.ready())
    capture_with(gc, graph_, s, [&](hipStream_t cs) {
      if (!batched) {  // one 8-byte all-reduce per integration
        for (int i = 0; i < graph_steps_; ++i) enqueue(cs);
        return;
      }
      // integration i's value -> outs[i]: mapped pinned memory on one rank, else the
      // device slots one all-reduce (+ one copy) closes
      double* outs = multi ? result_.get() : host_.device_ptr();
      if (row1_ <= row0_) {  // more ranks than rows
        MIINT_HIP(hipMemsetAsync(outs, 0, graph_steps_ * sizeof(double), cs));
      } else if (multistep()) {  // one launch for the replay's integrations + one close
        const int n = static_cast<int>(oracle::profile_table().size());
        const Table2DParams p{table_.get(), n, n, cfg_.extent, cfg_.extent, cfg_.grid,
                              cfg_.grid, row0_, row1_, cfg_.min_wg};
        launch_table2d_multistep(p, ms_partials_.get(), graph_steps_, outs, cs, phases_);
      } else if (chained()) {
        // integration i runs on chain i % L as that chain's step i / L: launch j of a chain
        // closes the chain's launch j - 1 (its workgroup 0), a finalize closes each chain,
        // and the plan's stream joins them all
        const int n = static_cast<int>(oracle::profile_table().size());
        const Table2DParams p{table_.get(), n, n, cfg_.extent, cfg_.extent, cfg_.grid,
                              cfg_.grid, row0_, row1_, cfg_.min_wg};
        const size_t nb = partials_.size();
        const int L = 1 + static_cast<int>(lanes_.size());
        auto lane = [&](int l) { return l == 0 ? cs : lanes_[static_cast<size_t>(l - 1)].get(); };
        auto half = [&](int l, int j) {
          return chain_.get() + (2 * static_cast<size_t>(l) + static_cast<size_t>(j & 1)) * nb;
        };
        if (L > 1) {
          ev_fork_.record(cs);
          for (int l = 1; l < L; ++l) MIINT_HIP(hipStreamWaitEvent(lane(l), ev_fork_.get(), 0));
        }
        for (int i = 0; i < graph_steps_; ++i) {
          const int l = i % L, j = i / L;
          launch_table2d_chained(p, half(l, j), j ? half(l, j - 1) : nullptr,
                                 j ? outs + i - L : nullptr, lane(l));
        }
        for (int l = 0; l < L; ++l) {
          const int last = l + ((graph_steps_ - 1 - l) / L) * L;
          launch_table2d_finalize(half(l, last / L), static_cast<int>(nb), outs + last, lane(l));
          if (l > 0) {
            ev_join_[static_cast<size_t>(l - 1)]->record(lane(l));
            MIINT_HIP(hipStreamWaitEvent(cs, ev_join_[static_cast<size_t>(l - 1)]->get(), 0));
          }
        }
      } else {
        for (int i = 0; i < graph_steps_; ++i) launch_local(outs + i, cs);
      }
      if (multi) {
        comm_->allreduce_sum(result_.get(), result_.get(), graph_steps_, cs);
        MIINT_HIP(hipMemcpyAsync(host_.get(), result_.get(), graph_steps_ * sizeof(double),
                                 hipMemcpyDeviceToHost, cs));
      }
    });
  const int launches = std::max(1, (iters + graph_steps_ - 1) / graph_steps_);
  // Warm-up: from idle the GPU needs ~25 ms of continuous work to reach steady clocks
  // (profiles/r1/clock_ramp.jsonl) and one replay here is 0.1-0.3 ms, so replay for about
  // cfg_.settle_ms first. Every replay of a collective plan holds collectives, so the count must
  // be the same on every rank: it comes from the plan's size (an estimate of the replay
  // time: ~0.5 ps per sample, >= 3 us per integration), not from a measurement.
  const double samples = static_cast<double>(cfg_.grid) * cfg_.grid / world_;
  const double est_replay_ms = graph_steps_ * std::max(3e-3, samples * 5e-10);
  const int warm = std::max(1, static_cast<int>(cfg_.settle_ms / est_replay_ms));
  for (int i = 0; i < warm; ++i) launch_with(gc, graph_, s);
  stream_.sync();
  barrier();
  e0_.record(s);
  for (int i = 0; i < launches; ++i) launch_with(gc, graph_, s);
  fault::delay(rank_);
  e1_.record(s);
  stream_.sync();
  last_batched_ = batched;
  return Event::elapsed_ms(e0_, e1_) / (launches * graph_steps_);
}

double Table2DPlan::last_result() const {
  return last_batched_ ? host_[graph_steps_ - 1] : host_[0];
}

int table2d_auto_graph_steps(int grid, double extent, int world) {
  MIINT_CHECK(grid >= 1 && world >= 1, "table2d: grid and world >= 1");
  const int n = static_cast<int>(oracle::profile_table().size());
  const int rows = (grid + world - 1) / world;  // the largest rank's rows
  // (num_cus is not consulted: the row-stream shape needs no residency)
  if (!table2d_multistep_ok(Table2DParams{nullptr, n, n, extent, extent, grid, grid, 0, rows, 1},
                            0))
    return Table2DPlan::kGraphSteps;
  const double samples = static_cast<double>(grid) * rows;
  int steps = Table2DPlan::kGraphSteps;
  while (steps < kT2MaxReplaySteps && steps * samples < Table2DPlan::kReplaySamples) steps *= 2;
  return steps;
}

double table2d_oracle(int grid, double extent) {
  const auto& v = oracle::profile_table();
  const double dx = extent / grid;
  const double cells = static_cast<double>(v.size() - 1) / extent;
  long double s = 0.0L;
  for (int j = 0; j < grid; ++j) s += oracle::interp(v, ((j + 0.5) * dx) * cells);
  const long double one = s * dx;
  return static_cast<double>(one * one);
}

}  // namespace miint
