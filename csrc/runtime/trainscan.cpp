// TrainScan implementation (see miint/trainscan.hpp).
#include "miint/trainscan.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "miint/fault.hpp"
#include "miint/integrator.hpp"
#include "miint/kernels.hpp"
#include "miint/oracle.hpp"
#include "miint/trace.hpp"

namespace miint {

namespace {
// scratch_ layout
constexpr int kLocalTotal = 0;  // [0] look-back: local slice total
constexpr int kCarry = 1;       // [1] look-back carry | [2..3] fused {C1, C2}
constexpr int kPick = 4;        // [4] pick_global value
constexpr int kTotals = 5;      // [5..6] fused {T1, T2}, [7] count
constexpr int kParity = 8;      // [8..9] --parity serial {last, at}
constexpr int kFlag = 10;       // [10] timeout flag (all-reduced: ranks that timed out)
constexpr int kSync = 11;       // [11] barrier operand
constexpr int kGather = 12;     // [12 ..) gathered values (3 per rank)
}  // namespace

TrainScan::TrainScan(const TrainScanConfig& cfg, int device, const Comm* comm)
    : cfg_(cfg), device_(device), comm_(comm), stream_((set_device(device), Stream())) {
  if (comm) {
    rank_ = comm->rank();
    world_ = comm->world();
    MIINT_CHECK(comm->device() == device, "communicator bound to another device");
  }
  MIINT_CHECK(cfg.steps_per_sec >= 1 && cfg.seconds >= 1, "bad train-scan size");
  total_ = static_cast<uint64_t>(cfg.steps_per_sec) * static_cast<uint64_t>(cfg.seconds);
  if (cfg.parity) {
    // 4main.c:90 subrange = tablelen / comm_sz (residual never scanned), and
    // 4main.c:76-78 fill window = whole seconds floor(1800/P) per rank.
    const uint64_t sub = total_ / static_cast<uint64_t>(world_);
    begin_ = static_cast<uint64_t>(rank_) * sub;
    count_ = sub;
    const uint64_t fs = static_cast<uint64_t>(cfg.seconds / world_) * cfg.steps_per_sec;
    win_lo_ = static_cast<uint64_t>(rank_) * fs;
    win_hi_ = win_lo_ + fs;
  } else {
    rank_slice(total_, rank_, world_, &begin_, &count_);
  }
  MIINT_CHECK(count_ >= 1, "empty slice");
  const std::vector<double>& tab = cfg.table.empty() ? oracle::profile_table() : cfg.table;
  MIINT_CHECK(tab.size() >= 2 && tab.size() <= 2048, "train table needs 2..2048 entries");
  MIINT_CHECK(static_cast<size_t>(cfg.seconds) <= tab.size() - 1,
              "trainscan: seconds exceeds the table (" + std::to_string(tab.size() - 1) + " s)");
  tn_ = static_cast<int>(tab.size());
  table_ = DeviceBuffer<double>(tab.size());
  MIINT_HIP(hipMemcpy(table_.get(), tab.data(), table_.bytes(), hipMemcpyHostToDevice));
  vel_ = DeviceBuffer<double>(count_);
  if (cfg.algo == ScanAlgo::kOnePass && world_ > 1) cfg_.algo = ScanAlgo::kFused;  // needs totals first
  if (cfg.phase2 || cfg_.algo != ScanAlgo::kLookback) pos_ = DeviceBuffer<double>(count_);
  if (cfg.replicate) {
    MIINT_CHECK(!cfg.parity && total_ % static_cast<uint64_t>(world_) == 0,
                "replicate needs equal slices (total divisible by world, no parity)");
    full_ = DeviceBuffer<double>(total_);
  }
  state_ = DeviceBuffer<char>(cfg_.algo == ScanAlgo::kLookback ? scan_state_bytes(count_)
                                                               : trainscan_workspace_bytes(count_));
  scratch_ = DeviceBuffer<double>(kGather + 3 * static_cast<size_t>(world_));  // >= 2 per rank
  host_ = PinnedBuffer<double>(4);
  MIINT_HIP(hipMemset(scratch_.get(), 0, scratch_.bytes()));
  MIINT_HIP(hipMemset(state_.get(), 0, state_.bytes()));
  const double cnt = static_cast<double>(count_);
  MIINT_HIP(hipMemcpy(scratch_.get() + kTotals + 2, &cnt, sizeof(double), hipMemcpyHostToDevice));
  MIINT_HIP(hipDeviceSynchronize());
}

// Look-back path: replace this rank's locally scanned slice by the globally scanned one —
// allgather every rank's local total, form the exclusive carry, add it in place.
void TrainScan::exchange_carry(const double* slice, uint64_t n, double* slice_out,
                               hipStream_t s) {
  if (!comm_ || world_ == 1) return;
  double* sc = scratch_.get();
  MIINT_HIP(hipMemcpyAsync(sc + kLocalTotal, slice + (n - 1), sizeof(double),
                           hipMemcpyDeviceToDevice, s));
  comm_->allgather(sc + kLocalTotal, sc + kGather, 1, s);
  launch_exclusive_carry(sc + kGather, rank_, sc + kCarry, s);
  if (rank_ > 0) launch_add_carry(slice_out, n, sc + kCarry, s);
}

// Value of global element `gi` (0 if no rank owns it, e.g. 4main's unscanned residual).
double TrainScan::pick_global(const double* slice, uint64_t gi, hipStream_t s) {
  double* sc = scratch_.get();
  MIINT_HIP(hipMemsetAsync(sc + kPick, 0, sizeof(double), s));
  if (gi >= begin_ && gi < begin_ + count_)
    MIINT_HIP(hipMemcpyAsync(sc + kPick, slice + (gi - begin_), sizeof(double),
                             hipMemcpyDeviceToDevice, s));
  if (comm_ && world_ > 1) comm_->allreduce_sum(sc + kPick, sc + kPick, 1, s);
  MIINT_HIP(hipMemcpyAsync(host_.get(), sc + kPick, sizeof(double), hipMemcpyDeviceToHost, s));
  MIINT_HIP(hipStreamSynchronize(s));
  return host_[0];
}

// --parity: the printed element exactly as 4main.c rounds it. Every rank runs the
// reference's sequential running sum over its slice (device, bit-exact), the {last, at}
// pairs meet in an allgather, and the root's carry fix-up (4main.c:147-154: block q adds
// the already-carried last element of block q-1, one fp64 add per element) is replayed in
// rank order: G_0 = last_0, G_q = last_q + G_{q-1}, element = at_q + G_{q-1}.
double TrainScan::parity_serial_element(uint64_t gi, hipStream_t s) {
  TrainScanKernelParams p{table_.get(), tn_,
                          1.0 / cfg_.steps_per_sec, begin_, count_, win_lo_, win_hi_};
  double* sc = scratch_.get();
  launch_trainscan_parity_serial(p, gi, sc + kParity, s);
  const int W = (comm_ && world_ > 1) ? world_ : 1;
  PinnedBuffer<double> h(2 * static_cast<size_t>(W));
  if (W > 1) {
    comm_->allgather(sc + kParity, sc + kGather, 2, s);
    MIINT_HIP(hipMemcpyAsync(h.get(), sc + kGather, 2 * W * sizeof(double), hipMemcpyDeviceToHost, s));
  } else {
    MIINT_HIP(hipMemcpyAsync(h.get(), sc + kParity, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  MIINT_HIP(hipStreamSynchronize(s));
  const uint64_t sub = count_;  // parity slices are all total / world long
  const uint64_t q = gi / sub;
  if (q >= static_cast<uint64_t>(W)) return 0.0;  // the unscanned residual (4main.c:91)
  double carry = 0.0;
  for (uint64_t b = 0; b < q; ++b) carry = b == 0 ? h[0] : h[2 * b] + carry;
  return q == 0 ? h[1] : h[2 * q + 1] + carry;
}

void TrainScan::enqueue_fused(hipStream_t s) {
  TrainScanKernelParams p{table_.get(), tn_,
                          1.0 / cfg_.steps_per_sec, begin_, count_, win_lo_, win_hi_};
  double* sc = scratch_.get();
  const bool fold = !(comm_ && world_ > 1);  // one GPU: no totals needed, no carries
  launch_trainscan_local(p, state_.get(), sc + kTotals, s, fold);
  const double* carries = nullptr;
  if (comm_ && world_ > 1) {
    // one {T1, T2, count} triple per rank (count written at construction), then each rank
    // forms its own carries
    comm_->allgather(sc + kTotals, sc + kGather, 3, s);
    launch_trainscan_rank_carry(sc + kGather, rank_, sc + kCarry + 1, s);
    carries = sc + kCarry + 1;
  }
  launch_trainscan_write(p, state_.get(), carries, vel_.get(), pos_.get(), s, fold);
}

void TrainScan::enqueue_onepass(hipStream_t s) {
  TrainScanKernelParams p{table_.get(), tn_,
                          1.0 / cfg_.steps_per_sec, begin_, count_, win_lo_, win_hi_};
  launch_trainscan_onepass(p, state_.get(), vel_.get(), pos_.get(), scratch_.get() + kTotals, s);
}

void TrainScan::enqueue_lookback(hipStream_t s) {
  const double dt = 1.0 / cfg_.steps_per_sec;
  const int tn = tn_;
  // Phase 1: velocity samples -> running integral (4main.c:95-160)
  launch_interp_scan_window(table_.get(), tn, dt, begin_, count_, win_lo_, win_hi_, vel_.get(),
                            state_.get(), nullptr, s);
  exchange_carry(vel_.get(), count_, vel_.get(), s);
  // Phase 2: running integral -> sum of sums (4main.c:178-221)
  if (cfg_.phase2) {
    launch_inclusive_scan(vel_.get(), pos_.get(), count_, state_.get(), nullptr, s);
    exchange_carry(pos_.get(), count_, pos_.get(), s);
  }
}

void TrainScan::enqueue() {
  DeviceGuard g(device_);
  TraceRange tr(cfg_.algo == ScanAlgo::kFused     ? "miint.trainscan.fused"
                : cfg_.algo == ScanAlgo::kOnePass ? "miint.trainscan.onepass"
                                                  : "miint.trainscan.lookback");
  hipStream_t s = stream_.get();
  if (cfg_.algo == ScanAlgo::kFused) enqueue_fused(s);
  else if (cfg_.algo == ScanAlgo::kOnePass) enqueue_onepass(s);
  else enqueue_lookback(s);
  if (cfg_.replicate) {
    if (comm_) {
      comm_->allgather(vel_.get(), full_.get(), count_, s);
    } else {
      MIINT_HIP(hipMemcpyAsync(full_.get(), vel_.get(), count_ * sizeof(double),
                               hipMemcpyDeviceToDevice, s));
    }
  }
}

ReplicaDigest digest_table(const double* host, uint64_t n) {
  ReplicaDigest d;
  d.n = n;
  uint64_t h = 1469598103934665603ull;  // FNV-1a 64
  double sum = 0.0, c = 0.0;            // Neumaier
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t bits;
    std::memcpy(&bits, &host[i], sizeof bits);
    for (int b = 0; b < 8; ++b) {
      h ^= (bits >> (8 * b)) & 0xffu;
      h *= 1099511628211ull;
    }
    const double x = host[i], t = sum + x;
    c += std::fabs(sum) >= std::fabs(x) ? (sum - t) + x : (x - t) + sum;
    sum = t;
  }
  d.hash = h;
  d.sum = sum + c;
  if (n > 0) {
    const uint64_t idx[5] = {0, n / 4, n / 2, 3 * (n / 4), n - 1};
    for (int k = 0; k < 5; ++k) d.at[k] = host[idx[k]];
  }
  return d;
}

ReplicaDigest TrainScan::replica_digest() {
  MIINT_CHECK(cfg_.replicate, "replica_digest needs --replicate");
  DeviceGuard g(device_);
  std::vector<double> h(total_);
  MIINT_HIP(hipMemcpyAsync(h.data(), full_.get(), total_ * sizeof(double), hipMemcpyDeviceToHost,
                           stream_.get()));
  MIINT_HIP(hipStreamSynchronize(stream_.get()));
  return digest_table(h.data(), total_);
}

TrainScanResult TrainScan::run() {
  DeviceGuard g(device_);
  hipStream_t s = stream_.get();
  TrainScanResult r;
  const bool multi = comm_ && world_ > 1;
  double* sc = scratch_.get();
  if (multi) {  // barrier: no rank's clock starts before every rank is here
    comm_->allreduce_sum(sc + kSync, sc + kSync, 1, s);
    wait_with_timeout(s, 300.0, comm_);
  }
  e0_.record(s);
  enqueue();
  fault::delay(rank_);
  e1_.record(s);
  MIINT_HIP(hipStreamSynchronize(s));
  r.device_ms = Event::elapsed_ms(e0_, e1_);
  if (cfg_.algo == ScanAlgo::kLookback) r.timeout = scan_timeout_flag(state_.get(), s);
  if (cfg_.algo == ScanAlgo::kOnePass) r.timeout = trainscan_onepass_timeout(state_.get(), s);
  if (cfg_.algo == ScanAlgo::kFused) {
    const TrainScanKernelParams p{table_.get(), tn_, 1.0 / cfg_.steps_per_sec, begin_, count_,
                                  win_lo_, win_hi_};
    r.timeout = trainscan_local_timeout(p, state_.get(), s);
  }
  if (fault::scan_timeout(rank_)) r.timeout = 1;  // MIINT_FAULT_*: the agreement tests
  r.timeout_ranks = r.timeout ? 1 : 0;
  if (multi) {  // a timeout on any rank is every rank's (before anyone enters another collective)
    host_[1] = r.timeout ? 1.0 : 0.0;
    MIINT_HIP(hipMemcpyAsync(sc + kFlag, host_.get() + 1, sizeof(double), hipMemcpyHostToDevice, s));
    comm_->allreduce_sum(sc + kFlag, sc + kFlag, 1, s);
    MIINT_HIP(hipMemcpyAsync(host_.get() + 1, sc + kFlag, sizeof(double), hipMemcpyDeviceToHost, s));
    wait_with_timeout(s, 300.0, comm_);
    r.timeout_ranks = static_cast<int>(host_[1]);
    r.timeout = r.timeout_ranks > 0 ? 1u : 0u;
  }
  // a look-back that gave up has poisoned its outputs with NaN: never hand them back
  if (r.timeout)
    throw ScanTimeout("trainscan: a hand-off spin hit its limit on " +
                      std::to_string(r.timeout_ranks) + " of " + std::to_string(world_) +
                      " rank(s) (a predecessor tile or block never published); results are "
                      "invalid",
                      r.timeout_ranks);
  // 4main.c:241 prints default_sum[tablelen-2]; the complete integral is element T-1.
  const uint64_t gi = cfg_.parity ? total_ - 2 : total_ - 1;
  r.distance = pick_global(vel_.get(), gi, s) / cfg_.steps_per_sec;
  r.distance_scan = r.distance;
  if (cfg_.parity) r.distance = parity_serial_element(gi, s) / cfg_.steps_per_sec;
  if (cfg_.phase2 || cfg_.algo != ScanAlgo::kLookback) {
    const uint64_t last = cfg_.parity ? (total_ / world_) * world_ - 1 : total_ - 1;
    r.sum_of_sums = pick_global(pos_.get(), last, s);
  }
  return r;
}

}  // namespace miint
