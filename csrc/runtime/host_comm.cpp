// HostComm: collectives between host processes over a TCP star (see miint/host.hpp).
//
// Replaces the reference's MPI point-to-point gathers (riemann.cpp:76-85: every worker
// MPI_Send's one double, rank 0 MPI_Recv's them in rank order and adds) and its
// MPI_Reduce / MPI_Bcast (4main.c:134-157) for the CPU path. Rank 0 accepts world - 1
// connections once (each peer first sends its rank); a reduction is: every rank sends its
// vector, rank 0 sums in rank order 0, 1, ..., world - 1 and sends the result back. Every
// receive polls with the communicator's timeout, so a dead peer fails the job.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "miint/common.hpp"
#include "miint/host.hpp"
#include "miint/net.hpp"
#include "miint/runtime.hpp"

namespace miint {

namespace {
void no_delay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
}  // namespace

HostComm::HostComm(const std::string& addr, int port, int rank, int world, double timeout_s)
    : rank_(rank), world_(world), timeout_s_(timeout_s) {
  MIINT_CHECK(world >= 1 && rank >= 0 && rank < world, "host comm: bad rank/world");
  if (world == 1) return;
  const double t0 = wall_seconds();
  if (rank == 0) {
    peers_.assign(world, -1);
    int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    MIINT_CHECK(srv >= 0, "host comm: socket()");
    int one = 1;
    ::setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(port));
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(srv, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) {
      ::close(srv);
      fail("host comm: bind failed on port " + std::to_string(port), __FILE__, __LINE__);
    }
    ::listen(srv, world);
    // any failure below closes the listener and every accepted peer before it propagates
    // (a constructor that throws runs no destructor)
    auto drop_all = [&] {
      ::close(srv);
      for (int& fd : peers_) {
        if (fd >= 0) ::close(fd);
        fd = -1;
      }
    };
    try {
      for (int got = 1; got < world; ++got) {
        pollfd pf{srv, POLLIN, 0};
        const double left = timeout_s - (wall_seconds() - t0);
        if (left <= 0 || ::poll(&pf, 1, static_cast<int>(left * 1e3) + 1) <= 0) {
          fail("host comm: " + std::to_string(got - 1) + " of " + std::to_string(world - 1) +
                   " ranks connected before the timeout",
               __FILE__, __LINE__);
        }
        const int c = ::accept(srv, nullptr, nullptr);
        MIINT_CHECK(c >= 0, "host comm: accept()");
        no_delay(c);
        int32_t who = -1;
        try {
          recv_from(c, &who, sizeof(who));
        } catch (...) {
          ::close(c);
          throw;
        }
        if (who < 1 || who >= world || peers_[who] >= 0) {
          ::close(c);
          fail("host comm: bad or duplicate rank " + std::to_string(who), __FILE__, __LINE__);
        }
        peers_[who] = c;
      }
    } catch (...) {
      drop_all();
      throw;
    }
    ::close(srv);
    return;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  MIINT_CHECK(::getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) == 0,
              "host comm: getaddrinfo(" + addr + ")");
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0 && !self_connected(fd)) {
      no_delay(fd);
      peers_.assign(1, fd);
      break;
    }
    if (fd >= 0) ::close(fd);
    if (wall_seconds() - t0 > timeout_s) {
      ::freeaddrinfo(res);
      fail("host comm: timed out connecting to rank 0 at " + addr + ":" + std::to_string(port),
           __FILE__, __LINE__);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  ::freeaddrinfo(res);
  const int32_t me = rank;
  try {
    send_to(peers_[0], &me, sizeof(me));
  } catch (...) {
    ::close(peers_[0]);
    throw;
  }
}

HostComm::~HostComm() {
  for (int fd : peers_)
    if (fd >= 0) ::close(fd);
}

void HostComm::send_to(int fd, const void* p, size_t bytes) {
  const char* c = static_cast<const char*>(p);
  while (bytes) {
    const ssize_t k = ::send(fd, c, bytes, MSG_NOSIGNAL);
    if (k <= 0) fail("host comm: send failed (peer gone?)", __FILE__, __LINE__);
    c += k;
    bytes -= static_cast<size_t>(k);
  }
}

void HostComm::recv_from(int fd, void* p, size_t bytes) {
  char* c = static_cast<char*>(p);
  const double t0 = wall_seconds();
  while (bytes) {
    pollfd pf{fd, POLLIN, 0};
    const double left = timeout_s_ - (wall_seconds() - t0);
    if (left <= 0 || ::poll(&pf, 1, static_cast<int>(left * 1e3) + 1) <= 0)
      fail("host comm: rank " + std::to_string(rank_) + " timed out waiting for a peer",
           __FILE__, __LINE__);
    const ssize_t k = ::recv(fd, c, bytes, 0);
    if (k <= 0) fail("host comm: peer closed the connection", __FILE__, __LINE__);
    c += k;
    bytes -= static_cast<size_t>(k);
  }
}

void HostComm::allreduce_sum(double* v, size_t n) {
  if (world_ == 1) return;
  const size_t bytes = n * sizeof(double);
  if (rank_ != 0) {
    send_to(peers_[0], v, bytes);
    recv_from(peers_[0], v, bytes);
    return;
  }
  std::vector<double> in(n);
  for (int q = 1; q < world_; ++q) {  // rank order: v = ((v0 + v1) + v2) + ...
    recv_from(peers_[q], in.data(), bytes);
    for (size_t i = 0; i < n; ++i) v[i] += in[i];
  }
  for (int q = 1; q < world_; ++q) send_to(peers_[q], v, bytes);
}

void HostComm::allgather(const double* send, double* recv, size_t n) {
  const size_t bytes = n * sizeof(double);
  std::memmove(recv + static_cast<size_t>(rank_) * n, send, bytes);
  if (world_ == 1) return;
  if (rank_ != 0) {
    send_to(peers_[0], send, bytes);
    recv_from(peers_[0], recv, bytes * world_);
    return;
  }
  for (int q = 1; q < world_; ++q) recv_from(peers_[q], recv + static_cast<size_t>(q) * n, bytes);
  for (int q = 1; q < world_; ++q) send_to(peers_[q], recv, bytes * world_);
}

void HostComm::broadcast(double* v, size_t n, int root) {
  MIINT_CHECK(root >= 0 && root < world_, "host comm: broadcast root out of range");
  if (world_ == 1) return;
  const size_t bytes = n * sizeof(double);
  if (rank_ == 0) {
    if (root != 0) recv_from(peers_[root], v, bytes);
    for (int q = 1; q < world_; ++q)
      if (q != root) send_to(peers_[q], v, bytes);
    return;
  }
  if (rank_ == root) send_to(peers_[0], v, bytes);
  else recv_from(peers_[0], v, bytes);
}

void HostComm::barrier() {
  double z = 0.0;
  allreduce_sum(&z, 1);
}

}  // namespace miint
