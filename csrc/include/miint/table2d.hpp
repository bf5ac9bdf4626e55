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
  // Without a communicator: integrate only row slice `rank` of `world` (the share one GPU
  // of a `world`-GPU run computes; the result is that partial). Ignored with a communicator.
  int world = 1, rank = 0;
  // Graph timing with a communicator: the kGraphSteps integrations of one replay each write
  // their own partial, and ONE all-reduce of kGraphSteps doubles (plus one copy) ends the
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
  // kGraphSteps integrations are captured once into a hipGraph and replayed (iters rounded
  // up to whole replays): one launch per kGraphSteps instead of one per integration.
  double time(int iters, bool graphs = true);
  // Global value of the last integration time() ran (every rank holds it).
  double last_result() const;
  bool bucketed() const { return bucketed_; }
  bool chained() const { return cfg_.chain && (!comm_ || world_ == 1 || bucketed_); }
  static constexpr int kGraphSteps = 32;
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
  DeviceBuffer<double> ms_partials_;  // multistep: kGraphSteps x workgroups
  int device_;
  const Comm* comm_;
  int rank_ = 0, world_ = 1;
  int row0_ = 0, row1_ = 0;
  bool bucketed_ = false;
  bool last_batched_ = false;  // the last time() left kGraphSteps results in host_
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

// Host oracle for the midpoint sum on a g x g grid: (sum_j v(x_j) dx)^2.
double table2d_oracle(int grid, double extent = 1800.0);

}  // namespace miint
