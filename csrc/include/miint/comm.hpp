// RCCL communicator wrapper (collectives over xGMI between the GPUs of one node).
//
// Replaces every MPI call site of the reference:
//   riemann.cpp:76,82-85   worker MPI_Send + root MPI_Recv loop  -> allreduce_sum(1 x f64)
//   4main.c:134,200        MPI_Reduce of local sums              -> allreduce_sum
//   4main.c:141-157        slice gather to root + serial carry + 144 MB Bcast
//                          -> allgather of P block totals (P x 8 B) + on-device carry add;
//                             optional allgather of the full table when every rank needs it
//   4main.c:137 Barrier    -> stream order (or a 0-byte-equivalent allreduce)
// Two bootstrap modes: one process per GPU (unique id exchanged out of band, e.g. through
// torch.distributed's store or miint's TCP rendezvous) and one process driving all GPUs
// (ncclCommInitAll). Collectives are enqueued on the caller's stream so they can be
// captured into a hipGraph together with the kernels that feed them.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <memory>
#include <string>
#include <vector>

#include "miint/common.hpp"

#define MIINT_RCCL(expr)                                                                 \
  do {                                                                                   \
    ncclResult_t miint_r_ = (expr);                                                      \
    if (miint_r_ != ncclSuccess)                                                         \
      ::miint::fail(std::string(#expr) + " -> " + ncclGetErrorString(miint_r_), __FILE__, \
                    __LINE__);                                                           \
  } while (0)

namespace miint {

class Comm {
 public:
  // 128-byte RCCL unique id (raw bytes), created by rank 0 and shared out of band.
  static std::string unique_id();
  // One process per GPU.
  Comm(const std::string& id, int rank, int world, int device);
  // One process, all listed devices (rank i <-> devices[i]).
  static std::vector<std::unique_ptr<Comm>> init_all(const std::vector<int>& devices);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }

  void allreduce_sum(const double* send, double* recv, size_t count, hipStream_t s) const;
  void allgather(const double* send, double* recv, size_t count_per_rank, hipStream_t s) const;
  void broadcast(double* buf, size_t count, int root, hipStream_t s) const;
  void reduce_sum(const double* send, double* recv, size_t count, int root, hipStream_t s) const;
  // Throws if RCCL reported an asynchronous error (e.g. a peer died).
  void check_async() const;
  // Abort outstanding collectives (watchdog path); the communicator is unusable afterwards.
  void abort() const;

  static void group_start();
  static void group_end();
  static std::string version();

 private:
  Comm() = default;
  mutable ncclComm_t comm_ = nullptr;  // nulled by abort()
  int rank_ = 0, world_ = 1, device_ = 0;
};

// Minimal TCP rendezvous for native multi-process launches (no MPI in the image, and the
// CLI must not depend on Python): rank 0 listens on addr:port and hands the RCCL unique id
// to every other rank. Used when the CLI is launched by torchrun --no-python.
std::string rendezvous_unique_id(const std::string& addr, int port, int rank, int world,
                                 double timeout_s = 120.0);
// The transport underneath: rank 0 serves `payload` (exactly len bytes) to world - 1
// connections and returns it; every other rank connects (retrying until rank 0 listens)
// and returns the len bytes it received. Both sides fail after timeout_s.
std::string rendezvous_share(const std::string& addr, int port, int rank, int world,
                             const std::string& payload, size_t len, double timeout_s);

}  // namespace miint
