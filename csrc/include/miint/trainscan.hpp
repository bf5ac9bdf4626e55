// Train-profile prefix-scan pipeline: the MI355X-native form of 4main.c.
//
// 4main.c: every rank interpolates its seconds of the 1801-point
// velocity profile at 1e4 samples/s into a private 144 MB array, scans a *different*
// element partition, ships every slice to rank 0, which adds carries serially and
// broadcasts the 144 MB table; then does it all again for the second integral.
//
// Here, per rank (one GPU):
//   phase 1  fused interp+scan kernel (decoupled look-back) -> velocity-integral slice
//            allgather of one fp64 slice total per rank -> exclusive carry -> add
//   phase 2  scan of the phase-1 slice -> position slice, same carry exchange
//   optional allgather of the full tables (the reference's "every rank has the table").
// Communication volume: 2 x world x 8 B instead of 2 x (gather + broadcast) of 144 MB.
// --parity reproduces 4main's partitions (fill by seconds, scan by elements, residual
// never scanned, value printed from element T-2), so P=7 prints 0 and P=16 117642.707174.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "miint/comm.hpp"
#include "miint/runtime.hpp"

namespace miint {

struct TrainScanConfig {
  int steps_per_sec = 10000;  // 4main.c:26
  int seconds = 1800;         // 4main.c:27 (table covers 1800 s)
  bool parity = false;        // emulate 4main.c partitions and printed element
  bool replicate = false;     // allgather full tables to every rank (4main.c:157)
  bool phase2 = true;         // second integral (4main.c:178-221)
};

struct TrainScanResult {
  double distance = 0.0;     // phase-1 value "Total distance traveled" (already / sps)
  double sum_of_sums = 0.0;  // phase-2 last scanned element (raw, not scaled)
  double device_ms = 0.0;
  unsigned timeout = 0;      // look-back spin gave up (never expected)
};

class TrainScan {
 public:
  TrainScan(const TrainScanConfig& cfg, int device, const Comm* comm = nullptr);
  TrainScanResult run();
  uint64_t total() const { return total_; }
  uint64_t local_begin() const { return begin_; }
  uint64_t local_count() const { return count_; }
  const double* velocity() const { return vel_.get(); }
  const double* position() const { return pos_.get(); }
  const double* replicated() const { return full_.get(); }

 private:
  void exchange_carry(const double* slice, uint64_t n, double* slice_out, hipStream_t s);
  double pick_global(const double* slice, uint64_t global_index, hipStream_t s);

  TrainScanConfig cfg_;
  int device_;
  const Comm* comm_;
  int rank_ = 0, world_ = 1;
  uint64_t total_ = 0, begin_ = 0, count_ = 0;
  uint64_t win_lo_ = 0, win_hi_ = ~uint64_t(0);
  Stream stream_;
  DeviceBuffer<double> table_, vel_, pos_, full_;
  DeviceBuffer<char> state_;
  DeviceBuffer<double> scratch_;  // [0] local total, [1] carry, [2] pick, [8..8+world) totals
  PinnedBuffer<double> host_;
  Event e0_, e1_;
};

// Exclusive carry for `rank` from the gathered per-rank totals (fixed order).
void launch_exclusive_carry(const double* totals, int rank, double* out, hipStream_t s);

}  // namespace miint
