// Communicators (RCCL, loopback) + TCP unique-id rendezvous (see miint/comm.hpp).
#include "miint/comm.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "miint/net.hpp"
#include "miint/runtime.hpp"

namespace miint {

bool ranks_share_devices() {
  const char* v = std::getenv("MIINT_OVERSUBSCRIBE");
  return v && std::strcmp(v, "0") != 0 && *v != '\0';
}

int rank_device(int local_rank) {
  if (!ranks_share_devices()) return local_rank;
  const int nd = device_count();
  MIINT_CHECK(nd >= 1, "MIINT_OVERSUBSCRIBE: no HIP devices visible");
  return local_rank % nd;
}

void prepare_shared_device_rccl(int rank) {
  if (!ranks_share_devices()) return;
  ::setenv("NCCL_SOCKET_IFNAME", "lo", 0);  // the ranks are on this host
  ::setenv("NCCL_IB_DISABLE", "1", 0);
  if (rank >= 0) ::setenv("NCCL_HOSTID", ("miint-shared-rank-" + std::to_string(rank)).c_str(), 1);
}

std::string RcclComm::unique_id() {
  capture_rccl_log();  // before the process's first RCCL call (RCCL reads its env once)
  prepare_shared_device_rccl(-1);
  ncclUniqueId id;
  MIINT_RCCL(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& id, int rank, int world, int device)
    : Comm(rank, world, device) {
  MIINT_CHECK(id.size() == sizeof(ncclUniqueId), "unique id must be 128 bytes");
  MIINT_CHECK(rank >= 0 && rank < world, "rank out of range");
  ncclUniqueId uid;
  std::memcpy(&uid, id.data(), sizeof(uid));
  capture_rccl_log();
  prepare_shared_device_rccl(rank);
  DeviceGuard g(device);
  MIINT_RCCL(ncclCommInitRank(&comm_, world, uid, rank));
}

std::vector<std::unique_ptr<Comm>> RcclComm::init_all(const std::vector<int>& devices) {
  const int n = static_cast<int>(devices.size());
  MIINT_CHECK(n >= 1, "need at least one device");
  capture_rccl_log();
  std::vector<ncclComm_t> comms(n);
  MIINT_RCCL(ncclCommInitAll(comms.data(), n, devices.data()));
  std::vector<std::unique_ptr<Comm>> out;
  for (int i = 0; i < n; ++i) out.emplace_back(new RcclComm(comms[i], i, n, devices[i]));
  return out;
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(comm_);
}

int RcclComm::transport_world() const {
  MIINT_CHECK(comm_ != nullptr, "communicator aborted");
  int n = 0;
  MIINT_RCCL(ncclCommCount(comm_, &n));
  return n;
}

void RcclComm::allreduce_sum(const double* send, double* recv, size_t count, hipStream_t s) const {
  MIINT_RCCL(ncclAllReduce(send, recv, count, ncclFloat64, ncclSum, comm_, s));
}
void RcclComm::allgather(const double* send, double* recv, size_t count, hipStream_t s) const {
  MIINT_RCCL(ncclAllGather(send, recv, count, ncclFloat64, comm_, s));
}
void RcclComm::broadcast(double* buf, size_t count, int root, hipStream_t s) const {
  MIINT_RCCL(ncclBroadcast(buf, buf, count, ncclFloat64, root, comm_, s));
}
void RcclComm::reduce_sum(const double* send, double* recv, size_t count, int root,
                          hipStream_t s) const {
  MIINT_RCCL(ncclReduce(send, recv, count, ncclFloat64, ncclSum, root, comm_, s));
}
void RcclComm::check_async() const {
  MIINT_CHECK(comm_ != nullptr, "communicator aborted");
  ncclResult_t r = ncclSuccess;
  MIINT_RCCL(ncclCommGetAsyncError(comm_, &r));
  MIINT_RCCL(r);
}
void RcclComm::abort() const {
  if (comm_) (void)ncclCommAbort(comm_);
  comm_ = nullptr;
}
void RcclComm::group_start() { MIINT_RCCL(ncclGroupStart()); }
void RcclComm::group_end() { MIINT_RCCL(ncclGroupEnd()); }
std::string RcclComm::version() {
  int v = 0;
  MIINT_RCCL(ncclGetVersion(&v));
  return std::to_string(v);
}

// ------------------------------------------------------------------ TCP rendezvous
namespace {

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}
bool recv_all(int fd, char* p, size_t n) {
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

}  // namespace

std::string rendezvous_unique_id(const std::string& addr, int port, int rank, int world,
                                 double timeout_s) {
  if (world == 1) return RcclComm::unique_id();
  return rendezvous_share(addr, port, rank, world, rank == 0 ? RcclComm::unique_id() : std::string(),
                          sizeof(ncclUniqueId), timeout_s);
}

std::string rendezvous_share(const std::string& addr, int port, int rank, int world,
                             const std::string& payload, size_t len, double timeout_s) {
  const size_t kLen = len;
  const double t0 = wall_seconds();
  if (rank == 0) {
    MIINT_CHECK(payload.size() == kLen, "rendezvous payload must be " + std::to_string(kLen) + " bytes");
    const std::string& id = payload;
    int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    MIINT_CHECK(srv >= 0, "socket()");
    int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(port));
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(srv, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) {
      ::close(srv);
      fail("rendezvous bind failed on port " + std::to_string(port), __FILE__, __LINE__);
    }
    ::listen(srv, world);
    for (int served = 1; served < world; ++served) {
      // wait for the next rank, but not forever: a rank that never starts must fail the job
      pollfd pf{srv, POLLIN, 0};
      const double left = timeout_s - (wall_seconds() - t0);
      if (left <= 0 || ::poll(&pf, 1, static_cast<int>(left * 1e3) + 1) <= 0) {
        ::close(srv);
        fail("rendezvous timed out: " + std::to_string(served - 1) + " of " +
                 std::to_string(world - 1) + " ranks connected",
             __FILE__, __LINE__);
      }
      int c = ::accept(srv, nullptr, nullptr);
      if (c < 0 || !send_all(c, id.data(), kLen)) {
        if (c >= 0) ::close(c);
        ::close(srv);
        fail("rendezvous accept/send failed", __FILE__, __LINE__);
      }
      ::close(c);
    }
    ::close(srv);
    return id;
  }
  // Non-zero ranks: retry until rank 0 listens.
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  MIINT_CHECK(::getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) == 0,
              "getaddrinfo(" + addr + ")");
  std::string id(kLen, '\0');
  for (;;) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    // (a self-connected socket is not rank 0: drop it and retry, net.hpp)
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0 && !self_connected(fd) &&
        recv_all(fd, &id[0], kLen)) {
      ::close(fd);
      break;
    }
    if (fd >= 0) ::close(fd);
    if (wall_seconds() - t0 > timeout_s) {
      ::freeaddrinfo(res);
      fail("rendezvous timed out waiting for rank 0", __FILE__, __LINE__);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  ::freeaddrinfo(res);
  return id;
}

}  // namespace miint
