// Train-profile prefix-scan pipeline: the MI355X-native form of 4main.c.
//
// 4main.c: every rank interpolates its seconds of the 1801-point
// velocity profile at 1e4 samples/s into a private 144 MB array, scans a *different*
// element partition, ships every slice to rank 0, which adds carries serially and
// broadcasts the 144 MB table; then does it all again for the second integral.
//
// Here, per rank (one GPU), three algorithms:
//   kFused (default)  reduce-then-scan on the *computed* samples (trainscan.hip): per-tile
//                     sums (compute only) -> one-workgroup tile prefix -> [allgather of one
//                     {T1, T2, count} triple per rank -> rank carries] -> one write-only pass
//                     that emits both the running integral and its running integral.
//                     HBM traffic: 16 B per sample, written once.
//   kOnePass          the same outputs in ONE pass: samples generated once, local two-level
//                     scan, decoupled look-back over the tile state {sum v, sum of local
//                     running integral}, write-only vel/pos. Measured slower on MI355X
//                     (103 us vs 66 us for 18e6 samples): each 33 KB-LDS workgroup (4 per CU)
//                     holds its slot through cross-XCD sc1 look-back round trips before it
//                     can write. With world > 1 the rank totals are needed first: kFused.
//   kLookback         the general single-pass decoupled look-back scan (scan.hip), used as
//                     phase-1 interp+scan and phase-2 scan, with an allgather + carry add per
//                     phase (48 B per sample of traffic).
// Communication volume either way: a few x world x 8 B instead of 2 x (gather + broadcast)
// of 144 MB. --parity reproduces 4main's partitions (fill by seconds, scan by elements,
// residual never scanned, printed element T-2), so P=7 prints 0 and P=16 117642.707174.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "miint/comm.hpp"
#include "miint/runtime.hpp"

namespace miint {

enum class ScanAlgo : int { kFused = 0, kLookback = 1, kOnePass = 2 };

struct TrainScanConfig {
  int steps_per_sec = 10000;  // 4main.c:26
  int seconds = 1800;         // 4main.c:27 (table covers 1800 s)
  bool parity = false;        // emulate 4main.c partitions and printed element
  bool replicate = false;     // allgather full tables to every rank (4main.c:157)
  bool phase2 = true;         // second integral (4main.c:178-221)
  ScanAlgo algo = ScanAlgo::kFused;
  // velocity table at 1 s spacing (empty: the built-in ex4vel.h profile); `seconds` must not
  // exceed its length - 1 (a user profile: --profile FILE, oracle::load_profile)
  std::vector<double> table;
};

struct TrainScanResult {
  double distance = 0.0;     // phase-1 value "Total distance traveled" (already / sps)
  double sum_of_sums = 0.0;  // phase-2 last scanned element (raw, not scaled)
  double distance_scan = 0.0;  // --parity: the printed element as the parallel scan rounds it
  double device_ms = 0.0;
  unsigned timeout = 0;      // look-back spin gave up (never expected)
  int timeout_ranks = 0;     // ranks whose scan reported it (agreed over the communicator)
};

// A hand-off spin hit its limit on at least one rank. Every rank of the communicator throws
// it together (the flag is all-reduced first), so no rank is left waiting in a collective
// for a peer that gave up; the CLI turns it into exit status 3 on every rank.
struct ScanTimeout : Error {
  ScanTimeout(const std::string& what, int ranks_timed_out) : Error(what), ranks(ranks_timed_out) {}
  int ranks = 0;  // how many ranks' scans gave up
};

// Kernel-level parameters of the fused pipeline (trainscan.hip).
struct TrainScanKernelParams {
  const double* table;  // device profile table
  int table_n;
  double dt;            // seconds per sample
  uint64_t i0;          // global index of this slice's first sample
  uint64_t n;           // samples in the slice
  uint64_t win_lo, win_hi;  // samples outside [win_lo, win_hi) are zero (parity fills)
};
// Workspace of the fused/one-pass kernels: must be zero-filled once at allocation (tickets
// live in it and every launch leaves them re-armed).
size_t trainscan_workspace_bytes(uint64_t n);
// K1 + K2: per-tile sums and tile prefixes into `ws`; totals[0..1] = {T1, T2} (device).
// fold = true (one GPU, no carries): when the slice has at most 64 blocks of 256 tiles, stop
// at the per-block aggregates and let launch_trainscan_write(fold = true) fold them per
// workgroup; totals are then NOT written. Both calls must pass the same `fold`.
void launch_trainscan_local(const TrainScanKernelParams& p, void* ws, double* totals,
                            hipStream_t s, bool fold = false);
// K3: rank carries {C1, C2} from world x {T1, T2, count} gathered triples.
void launch_trainscan_rank_carry(const double* gathered, int rank, double* carries,
                                 hipStream_t s);
// K4: write vel (running integral) and pos (its running integral); carries may be null.
void launch_trainscan_write(const TrainScanKernelParams& p, const void* ws, const double* carries,
                            double* vel, double* pos, hipStream_t s, bool fold = false);
// --parity: the reference's sequential running sum over this slice, bit-exact (one
// workgroup); out[0] = sum at the slice's last element, out[1] = at global element `want`
// (0 if the slice does not hold it).
void launch_trainscan_parity_serial(const TrainScanKernelParams& p, uint64_t want, double* out,
                                    hipStream_t s);
// One pass (K1 + K2 + K4 with a decoupled look-back): vel, pos and totals {T1, T2}.
void launch_trainscan_onepass(const TrainScanKernelParams& p, void* ws, double* vel, double* pos,
                              double* totals, hipStream_t s);
// Nonzero if a one-pass look-back spin gave up (reads the workspace header; synchronises).
unsigned trainscan_onepass_timeout(const void* ws, hipStream_t s);
// Nonzero if the closed-form K1 + K2 launch's block-aggregate hand-off gave up waiting (its
// totals are then NaN); 0 for the 3-kernel path. Synchronises.
unsigned trainscan_local_timeout(const TrainScanKernelParams& p, const void* ws, hipStream_t s);

// A host-side fingerprint of a replicated table (--replicate, 4main.c:157's "every rank holds
// the whole table"): FNV-1a over the fp64 bit patterns (equal on every rank iff the copies are
// bitwise equal), a compensated sum and samples at fixed fractions of the table (comparable
// to the one-GPU table within roundoff: the carries round differently from one scan).
struct ReplicaDigest {
  uint64_t hash = 0;
  uint64_t n = 0;
  double sum = 0.0;
  double at[5] = {0, 0, 0, 0, 0};  // elements 0, n/4, n/2, 3n/4, n-1
};
ReplicaDigest digest_table(const double* host, uint64_t n);

class TrainScan {
 public:
  TrainScan(const TrainScanConfig& cfg, int device, const Comm* comm = nullptr);
  TrainScanResult run();
  // Enqueue one complete pipeline on the plan's stream without synchronising.
  void enqueue();
  uint64_t total() const { return total_; }
  ScanAlgo algo() const { return cfg_.algo; }  // effective (kOnePass -> kFused when world > 1)
  uint64_t local_begin() const { return begin_; }
  uint64_t local_count() const { return count_; }
  const double* velocity() const { return vel_.get(); }
  const double* position() const { return pos_.get(); }
  const double* replicated() const { return full_.get(); }
  // Copy the replicated table to the host and fingerprint it (--replicate only; synchronises;
  // not part of any timed region)
  ReplicaDigest replica_digest();
  hipStream_t stream() const { return stream_.get(); }

 private:
  void enqueue_fused(hipStream_t s);
  void enqueue_onepass(hipStream_t s);
  void enqueue_lookback(hipStream_t s);
  void exchange_carry(const double* slice, uint64_t n, double* slice_out, hipStream_t s);
  double pick_global(const double* slice, uint64_t global_index, hipStream_t s);
  double parity_serial_element(uint64_t global_index, hipStream_t s);

  TrainScanConfig cfg_;
  int device_;
  const Comm* comm_;
  int rank_ = 0, world_ = 1;
  int tn_ = 0;  // table entries
  uint64_t total_ = 0, begin_ = 0, count_ = 0;
  uint64_t win_lo_ = 0, win_hi_ = ~uint64_t(0);
  Stream stream_;
  DeviceBuffer<double> table_, vel_, pos_, full_;
  DeviceBuffer<char> state_;      // look-back scan state or fused-pipeline workspace
  DeviceBuffer<double> scratch_;  // [0..11] scalars, [12..) gathered per-rank values
  PinnedBuffer<double> host_;
  Event e0_, e1_;
};

// Exclusive carry for `rank` from the gathered per-rank totals (fixed order).
void launch_exclusive_carry(const double* totals, int rank, double* out, hipStream_t s);

}  // namespace miint
