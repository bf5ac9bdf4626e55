// 2-D velocity-field integral (BASELINE.json config #5; no counterpart in the reference,
// whose data is the 1-D ex4vel.h profile).
//
// Field: F(x, y) = v(x) v(y) on [0, 1800]^2, materialised as the 1801 x 1801 fp64 outer
// product of the generated profile (25.9 MB, built on the device), integrated with a
// midpoint rule on a g x g sample grid using bilinear interpolation of the table. The
// kernel (table.hip) gives each workgroup 256 sample columns by 4 R sample rows, stages the
// table footprint of that block in LDS (2-D LDS tiling) and streams each wave down its R
// rows (coarse grids: a tile kernel reading the table from global memory). Ranks split the
// sample rows; the per-rank partials meet in one RCCL all-reduce.
//
// Oracle: bilinear interpolation of a separable product of piecewise-linear factors is
// exactly v(x) v(y), so the midpoint sum equals (sum_j v(x_j) dx)^2 — a 1-D computation —
// and the exact integral is 122000.004^2 = 1.4884000976e10.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "miint/comm.hpp"
#include "miint/kernels.hpp"
#include "miint/runtime.hpp"

namespace miint {

struct Table2DConfig {
  int grid = 4096;       // samples per axis
  double extent = 1800;  // [0, extent]^2
  // Without a communicator, or with a 1-rank one (force_collective): integrate only row
  // slice `rank` of `world` (the share one GPU of a `world`-GPU run computes; run() and
  // last_result() then return that slice's partial — a 1-rank all-reduce adds nothing).
  // Ignored with a communicator of more than one rank (its rank and world rule).
  int world = 1, rank = 0;
  // Graph timing with a communicator: the graph_steps integrations of one replay each write
  // their own partial, and ONE all-reduce of graph_steps doubles (plus one copy) ends the
  // replay — every integration still gets its own global sum (RiemannPlan's bucketing).
  // false: kernel -> 8-byte all-reduce -> copy per integration.
  bool bucket = true;
  // Graph timing: chained launches (launch j's workgroup 0 closes launch j-1's partials,
  // one finalize closes the replay) instead of the fused hand-off tail in every launch.
  bool chain = true;
  // Chained graph timing: the kGraphSteps integrations of a replay are dealt round-robin to
  // this many streams, each its own chain (integrations are independent: own partials, own
  // result), so one launch's staging latency and tail overlap the next one's work. 0 = auto
  // (kAutoT2Streams); 1 = one chain on the plan's stream.
  int step_streams = 0;
  // Chained graph timing as ONE multi-step launch of resident workgroups for the replay's
  // kGraphSteps integrations plus one closing kernel (launch_table2d_multistep): one launch
  // ramp and tail per replay. Used for every row-stream shape (resident or not); bitwise the
  // same values.
  bool multistep = true;
  // Multi-step step phases (launch_table2d_multistep): workgroups per row-stream block, each
  // running every phases-th integration of the replay; 0 = auto (kT2AutoPhases), 1 = one
  // workgroup per block (round 3's launch)
  int phases = 0;
  // row stream: fewest workgroups its shape aims for (0 = kernel default, 512 — except in a
  // multi-step plan, whose step phases supply the parallelism: there 0 means the most rows
  // per wave that fit the LDS tile, for every launch of the plan, so all its paths still
  // sum the same partials; 1/8 slice of 4096^2: 1.48 -> 1.23 us, profiles/r4/t2d_slice_shapes)
  int min_wg = 0;
  // Run the RCCL stage (the bucketed all-reduce + copy per replay) even with a 1-rank
  // communicator — a row slice (world/rank above) then times the per-GPU share of a
  // world-GPU run with its collective captured (tools/t2d_strong.py).
  bool force_collective = false;
  // Integrations per graph replay: 0 = auto (Table2DPlan::graph_steps), else 1..kT2MaxReplaySteps.
  int graph_steps = 0;
  double settle_ms = 30.0;  // graph time(): untimed warm-up replays first (steady clocks)
};
// 4096^2 on one MI355X, us per integration by chains 1/2/3/4/8 (two runs each, settled
// clocks; profiles/r3/t2d_streams.jsonl): whole field 8.51 / 6.7-6.9 / 7.1 / 7.5-7.6 / 7.3-7.5;
// a 1/8 row slice (the per-GPU share at 8 GPUs) 4.2 / 3.1-4.7 / 3.9-6.7 / 4.1-4.3 / 4.5-4.8.
constexpr int kAutoT2Streams = 2;

class Table2DPlan {
 public:
  Table2DPlan(const Table2DConfig& cfg, int device, const Comm* comm = nullptr);
  // One integration: one fused kernel (result straight into pinned host memory on one
  // rank) or kernel -> RCCL all-reduce -> 8-byte copy. Returns the value.
  double run();
  // `iters` back-to-back integrations; returns device ms per integration. With graphs,
  // graph_steps() integrations are captured once into a hipGraph and replayed (iters rounded
  // up to whole replays): one graph launch per graph_steps() integrations.
  double time(int iters, bool graphs = true);
  // Global value of the last integration time() ran (every rank holds it).
  double last_result() const;
  bool bucketed() const { return bucketed_; }
  bool chained() const { return cfg_.chain && (!collective_ || bucketed_); }
  // the replay ends in a collective over the plan's communicator (world > 1, or forced)
  bool collective() const { return collective_; }
  // Integrations per graph replay. Chained and per-launch replays: kGraphSteps (one kernel
  // node per integration). A multi-step replay (one launch + one close) under auto: doubled
  // from kGraphSteps until the replay holds kReplaySamples samples (<= kT2MaxReplaySteps) —
  // a replay pays ~14 us of launch ramp, tail and closing kernel whatever its size, which at
  // 32 integrations of a 1/8 row slice of 4096^2 (30 us of work) was a third of the time
  // (profiles/r5/t2d/n_t2d_steps.jsonl, us per integration at 32 / 128 / 512 / 1024 per
  // replay: 4096^2 4.61-4.71 / 4.34 / 4.12-4.20 / 4.12-4.16; its 1/8 slice 0.95-1.06 / 0.71-0.84
  // / 0.62 / 0.61-0.63). Every integration is still a complete one (its own staging and
  // partials), and every replay size gives the same values, bitwise.
  static constexpr int kGraphSteps = 32;
  static constexpr double kReplaySamples = 8589934592.0;  // 2^33: 512 integrations of 4096^2
  int graph_steps() const { return graph_steps_; }
  int step_streams() const;  // chains a chained replay runs (1 when not chained)
  // Collective over the plan's communicator (no-op on one rank): time() calls it right
  // before its clock starts, so every rank's interval begins after every rank is here.
  void barrier();
  // A chained replay is one multi-step launch (Table2DConfig::multistep, in effect).
  bool multistep() const { return chained() && multistep_; }
  int phases() const { return multistep() ? phases_ : 0; }  // step phases of a multi-step replay
  int resident_per_cu() const { return resident_per_cu_; }  // multi-step workgroups per CU
  int min_wg() const { return cfg_.min_wg; }  // the row-stream shape's target (after auto)
  int workgroups() const { return static_cast<int>(partials_.size()); }  // per integration
  int row0() const { return row0_; }
  int row1() const { return row1_; }

 private:
  void enqueue(hipStream_t s);
  void launch_local(double* out, hipStream_t s);  // this rank's rows -> *out (device ptr)
  Table2DConfig cfg_;
  bool multistep_ = false;
  int phases_ = 1;
  int resident_per_cu_ = 0;
  int graph_steps_ = kGraphSteps;
  DeviceBuffer<double> ms_partials_;  // multistep: graph_steps_ x workgroups
  int device_;
  const Comm* comm_;
  int rank_ = 0, world_ = 1;
  int row0_ = 0, row1_ = 0;
  bool bucketed_ = false;
  bool collective_ = false;
  bool last_batched_ = false;  // the last time() left graph_steps_ results in host_
  Stream stream_;
  std::vector<Stream> lanes_;  // streams 1.. of a multi-stream chained replay
  std::vector<std::unique_ptr<Event>> ev_join_;
  Event ev_fork_{false};
  DeviceBuffer<double> v_, table_, partials_, chain_, result_, sync_;
  DeviceBuffer<unsigned int> ticket_;
  PinnedBuffer<double> host_;
  Event e0_, e1_;
  Graph graph_;
};

// Auto integrations per multi-step replay (Table2DPlan::graph_steps) for a g x g grid whose
// rows are split over `world` ranks: from the configuration only — the largest rank's row
// count and whether that shape runs the row stream — so every rank of a collective plan
// replays the same count. kGraphSteps when the shape has no multi-step launch.
int table2d_auto_graph_steps(int grid, double extent, int world);

// Host oracle for the midpoint sum on a g x g grid: (sum_j v(x_j) dx)^2.
double table2d_oracle(int grid, double extent = 1800.0);

}  // namespace miint
