// Loopback rendezvous helpers shared by the RCCL unique-id rendezvous (comm.cpp), the host
// communicator (host_comm.cpp) and the launcher (miintrun.cpp).
//
// Two ways a localhost rendezvous port can be lost, both seen on the one-GPU pool when four
// ranks retry their connect() every 20 ms while rank 0 is still initialising:
//   * TCP self-connect: a connect() to 127.0.0.1:P with nobody listening on P can be given
//     the local ephemeral port P itself, and Linux then completes a "simultaneous open" with
//     itself. The rank believes it is connected (and waits forever for rank 0's bytes) while
//     rank 0's bind() of P fails (a rank-4 riemann run on the pool: "rendezvous bind failed").
//   * a launcher port taken from bind(0) lies INSIDE the ephemeral range, so it is exactly the
//     kind of port the retrying clients are handed as their local port.
// So clients drop self-connected sockets and retry, and the launcher picks its port below the
// ephemeral range.
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <initializer_list>
#include <random>

namespace miint {

// True if fd's local and peer addresses are the same (a TCP self-connect).
inline bool self_connected(int fd) {
  sockaddr_in a{}, b{};
  socklen_t la = sizeof(a), lb = sizeof(b);
  if (::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &la) != 0 ||
      ::getpeername(fd, reinterpret_cast<sockaddr*>(&b), &lb) != 0)
    return false;
  return a.sin_port == b.sin_port && a.sin_addr.s_addr == b.sin_addr.s_addr;
}

// Lowest port of the kernel's ephemeral (connect()) range; 32768 if unreadable.
inline int ephemeral_port_low() {
  int lo = 32768, hi = 60999;
  if (FILE* f = std::fopen("/proc/sys/net/ipv4/ip_local_port_range", "r")) {
    if (std::fscanf(f, "%d %d", &lo, &hi) != 2) lo = 32768;
    std::fclose(f);
  }
  return lo;
}

// A TCP port P such that P + o binds on every interface now for each offset o (the CLIs use
// MASTER_PORT + 17 for the RCCL unique id and + 19 for host collectives), all of them below
// the ephemeral range so no retrying client is handed one as its local port. Falls back to a
// kernel-chosen port.
inline int pick_rendezvous_port(std::initializer_list<int> offsets = {0}) {
  int span = 0;
  for (int o : offsets) span = o > span ? o : span;
  const int hi = ephemeral_port_low() - span;
  const int lo = hi > 21000 ? 20000 : 1024;
  auto bindable = [](int port, int* got) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return false;
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    sa.sin_port = htons(static_cast<uint16_t>(port));
    socklen_t len = sizeof(sa);
    const bool ok = ::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0 &&
                    ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len) == 0;
    if (ok && got) *got = ntohs(sa.sin_port);
    ::close(fd);
    return ok;
  };
  if (hi - 1 > lo) {
    std::random_device rd;
    std::mt19937 gen(rd());
    std::uniform_int_distribution<int> pick(lo, hi - 1);
    for (int tries = 0; tries < 64; ++tries) {
      const int p = pick(gen);
      bool ok = true;
      for (int o : offsets) ok = ok && bindable(p + o, nullptr);
      if (ok) return p;
    }
  }
  int got = 0;
  return bindable(0, &got) ? got : 29500;
}

}  // namespace miint
