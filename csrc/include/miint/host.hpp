// Host (CPU) execution: the "MPI" half of the reference's CUDA-vs-MPI comparison, native.
//
// The reference's riemann.cpp and 4main.c (C12-C15) are CPU programs: P
// MPI processes, each running a scalar fp64 loop over its slice (libm sin per sample,
// riemann.cpp:29-44; interpolate-then-scan, 4main.c:82-122), results gathered by
// point-to-point sends to rank 0. Here the same work runs as
//
//   HostPool      persistent worker threads of one process (the ranks of one node); every
//                 call splits its sample slice into balanced contiguous thread slices and
//                 combines the thread partials in thread order (deterministic for a fixed
//                 thread count).
//   host_riemann  the Riemann sum of every integrand over a sample slice, evaluated PER
//                 SAMPLE (IEEE division, a full sin/cos per sample, per-sample table
//                 interpolation — none of the GPU tile rewrites) in explicit 8-wide fp64
//                 vectors, built three times (AVX-512, AVX2+FMA, baseline x86-64) and
//                 dispatched on the CPU at run time.
//   HostComm      host collectives between PROCESSES (one per node or socket): a TCP star
//                 through rank 0 that sums in rank order, replacing MPI_Send/MPI_Recv
//                 (riemann.cpp:76-85) and MPI_Reduce/MPI_Bcast (4main.c:134-157).
//   host_trainscan the 4main.c pipeline on threads (and ranks): per-thread closed tile sums,
//                 an exclusive scan of the thread/rank totals, one write pass that emits the
//                 running integral and its running integral.
//
// It is what `--device cpu` runs in the native CLIs and `backend="host"` in Python, and the
// CPU column of `miint compare` (the reference's comparison, measured on one box).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "miint/integrator.hpp"

namespace miint {

class HostPool {
 public:
  // threads <= 0: MIINT_HOST_THREADS, else OMP_NUM_THREADS, else the CPUs in this process's
  // affinity mask (at least 1).
  explicit HostPool(int threads = 0);
  ~HostPool();
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;
  int threads() const { return n_; }
  static int default_threads();
  // fn(t) for every t in [0, threads()): t = 0 on the calling thread, the others on the
  // pool's workers. Returns when every call has returned; rethrows the first exception.
  void run(const std::function<void(int)>& fn);

 private:
  void worker(int t);
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  long gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  std::string err_;
};

// The vector ISA host_riemann dispatches to on this CPU: "avx512", "avx2" or "base".
const char* host_isa();

// h * scale * sum over samples [begin, begin + count) of cfg's n-sample rule on [a, b] (fp64,
// per-sample evaluation; cfg.dtype/div/grid are GPU knobs and ignored). Threads take
// balanced contiguous sub-slices; each accumulates 8 vector lanes over blocks of 4096
// samples and the block sums with compensation; thread partials are added in thread order.
double host_riemann(const RiemannConfig& cfg, uint64_t begin, uint64_t count, HostPool& pool);

// The reference's `mpirun -np P ./riemann` on P - 1 host threads, bit for bit: worker w
// runs riemann.cpp:29-44 (scalar libm sin, sequential fp64 sum, int counter) over
// [w R/W, (w+1) R/W) with (int)(n/W) samples, and the partials are added in rank order
// (riemann.cpp:82-85). Equals oracle::riemann_mpi_parity, which runs the workers serially.
double host_riemann_mpi_parity(int comm_size, double n, double range, HostPool& pool);

// A runtime integrand on the host: f(x) given as one C++ expression over x (the rules of
// expr_check, as for the GPU's hipRTC path), compiled by the system C++ compiler into a
// shared object (-O3 -march=native, scalar libm per sample, compensated blocks; compiler:
// MIINT_HOST_CXX, else /opt/rocm/llvm/bin/clang++, else c++) and dlopen'ed; cached per
// expression in the process.
class HostExpr {
 public:
  explicit HostExpr(const std::string& expr);
  // h * sum f(a + (i + off) h) over [begin, begin + count) of the n-sample rule on [a, b],
  // thread slices added in thread order.
  double integrate(double a, double b, uint64_t n, Rule rule, uint64_t begin, uint64_t count,
                   HostPool& pool) const;
  const std::string& expression() const { return expr_; }

 private:
  std::string expr_;
  void* fn_ = nullptr;
};

// Host collectives across processes: a TCP star through rank 0 (rank 0 listens on
// addr:port, every other rank connects once and keeps its socket). Reductions sum in rank
// order on rank 0, so every rank receives bitwise the same values. Every receive is bounded
// by timeout_s: a dead peer is an error, not a hang.
class HostComm {
 public:
  HostComm(const std::string& addr, int port, int rank, int world, double timeout_s = 120.0);
  ~HostComm();
  HostComm(const HostComm&) = delete;
  HostComm& operator=(const HostComm&) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  void allreduce_sum(double* v, size_t n);
  // recv holds world x n values in rank order.
  void allgather(const double* send, double* recv, size_t n);
  void broadcast(double* v, size_t n, int root);
  void barrier();

 private:
  void send_to(int fd, const void* p, size_t bytes);
  void recv_from(int fd, void* p, size_t bytes);
  int rank_, world_;
  double timeout_s_;
  std::vector<int> peers_;  // rank 0: socket of rank r at [r]; others: [0] = rank 0
};

struct HostScanConfig {
  int steps_per_sec = 10000;  // 4main.c:26
  int seconds = 1800;         // 4main.c:27
  bool keep = false;          // keep vel / pos (else only the totals are formed)
  std::vector<double> table;  // velocity table at 1 s spacing (empty: the built-in profile)
};
struct HostScanResult {
  double distance = 0.0;     // vel[T-1] / steps_per_sec (the complete running integral)
  double sum_of_sums = 0.0;  // pos[T-1]
  double seconds = 0.0;      // wall time of the pipeline (both passes + the carry exchange)
  uint64_t begin = 0, count = 0;  // this rank's slice of the T samples
};
// The 4main.c pipeline on this rank's slice (rank / world from comm, or 0 / 1): sample
// v_i = interp(profile, i / sps), vel = running sum of v, pos = running sum of vel. Pass 1:
// per-thread totals {sum v, sum of the thread's own running sums}; exclusive scan over
// threads and (allgather) ranks; pass 2 writes vel / pos with the carries (if keep) and the
// last element's values. vel / pos, when kept, are the slice's (count values each).
HostScanResult host_trainscan(const HostScanConfig& cfg, HostPool& pool, HostComm* comm,
                              std::vector<double>* vel = nullptr,
                              std::vector<double>* pos = nullptr);

}  // namespace miint
