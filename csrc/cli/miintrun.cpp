// miintrun — the `mpirun -np P` of this framework: start P ranks of a program, one process
// each, and wait for them (the reference launches riemann and 4main with Intel MPI's mpirun,
// riemann.cpp:62-64, 4main.c:69-71; there is no MPI in this image).
//
//   miintrun -np P [--addr 127.0.0.1] [--port 0] [--grace 10] [--linger 2] [--] PROGRAM [ARGS...]
//
// Every rank gets RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR and MASTER_PORT
// (a free port when --port 0), the environment torchrun gives and the native CLIs, bench.py
// and the Python package read: GPU ranks bootstrap RCCL from it, --device cpu ranks their
// host collectives. The first rank that fails (non-zero exit or a signal) ends the others
// (SIGTERM, SIGKILL after --grace seconds, to each rank's process group, so a rank's own
// children go too) and its status is miintrun's; SIGINT / SIGTERM are forwarded. A rank
// that EXITS with a status (rather than dying of a signal) first gives the others --linger
// seconds to finish on their own: a failure the ranks agreed on (every rank exits 3 after a
// scan timeout anywhere) then ends with rank 0's record printed, not cut off. This
// process links no HIP and touches no GPU, so starting programs from it is safe; ranks are
// started with fork + exec before anything in them has run.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "miint/net.hpp"

namespace {

volatile sig_atomic_t g_signal = 0;
void on_signal(int s) { g_signal = s; }

int usage(FILE* out = stderr) {
  std::fprintf(out,
               "usage: miintrun -np P [--addr A] [--port N] [--grace S] [--linger S] [--] "
               "PROGRAM [ARGS...]\n");
  return out == stderr ? 2 : 0;
}

int status_code(int st) { return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st); }

}  // namespace

int main(int argc, char** argv) {
  int np = 0, port = 0;
  double grace = 10.0, linger = 2.0;
  std::string addr = "127.0.0.1";
  int i = 1;
  for (; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "miintrun: %s needs a value\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "-h" || a == "--help") return usage(stdout);
    if (a == "-np" || a == "-n" || a == "--np") np = std::atoi(val("-np"));
    else if (a == "--addr") addr = val("--addr");
    else if (a == "--port") port = std::atoi(val("--port"));
    else if (a == "--grace") grace = std::atof(val("--grace"));
    else if (a == "--linger") linger = std::atof(val("--linger"));
    else if (a == "--") { ++i; break; }
    else if (!a.empty() && a[0] == '-') {
      std::fprintf(stderr, "miintrun: unknown option %s\n", a.c_str());
      return usage();
    } else break;
  }
  if (np < 1 || i >= argc) return usage();
  if (port == 0) port = miint::pick_rendezvous_port({0, 17, 19});  // + the CLIs' offsets (net.hpp)

  struct sigaction sa{};
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);

  std::vector<pid_t> pids(np, -1);
  for (int r = 0; r < np; ++r) {
    const pid_t pid = ::fork();
    if (pid < 0) {
      std::perror("miintrun: fork");
      for (int q = 0; q < r; ++q) ::kill(pids[q], SIGTERM);
      return 1;
    }
    if (pid == 0) {
      ::setpgid(0, 0);  // each rank its own process group: stopping a rank stops its children
      signal(SIGINT, SIG_DFL);
      signal(SIGTERM, SIG_DFL);
      const std::string R = std::to_string(r), W = std::to_string(np), P = std::to_string(port);
      setenv("RANK", R.c_str(), 1);
      setenv("LOCAL_RANK", R.c_str(), 1);
      setenv("WORLD_SIZE", W.c_str(), 1);
      setenv("LOCAL_WORLD_SIZE", W.c_str(), 1);
      setenv("MASTER_ADDR", addr.c_str(), 1);
      setenv("MASTER_PORT", P.c_str(), 1);
      ::execvp(argv[i], argv + i);
      std::fprintf(stderr, "miintrun: cannot run %s: %s\n", argv[i], std::strerror(errno));
      std::_Exit(127);
    }
    ::setpgid(pid, pid);  // (also here: no race with the first signal_all)
    pids[r] = pid;
  }

  int rc = 0, left = np;
  bool stopping = false, lingering = false;
  auto t_stop = std::chrono::steady_clock::now();
  auto t_linger = t_stop;
  auto since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
  };
  auto signal_all = [&](int sig) {  // every live rank's whole process group
    for (pid_t p : pids)
      if (p > 0) ::kill(-p, sig);
  };
  while (left > 0) {
    int st = 0;
    const pid_t p = ::waitpid(-1, &st, WNOHANG);
    if (p > 0) {
      for (auto& q : pids)
        if (q == p) q = -1;
      --left;
      const int code = status_code(st);
      if (code != 0 && rc == 0) {
        rc = code;
        std::fprintf(stderr, "miintrun: a rank exited with %d; stopping the others\n", code);
      }
      if (code != 0 && !stopping && WIFEXITED(st) && linger > 0) {
        // an exit status: the peers may be finishing the same agreed failure (every rank
        // exits 3 after a scan timeout anywhere). The first one starts the linger; further
        // exits with a status during it only set rc — stopping now could cut rank 0 off
        // before it prints its record, which is what the linger is for.
        if (!lingering) {
          lingering = true;
          t_linger = std::chrono::steady_clock::now();
        }
      } else if (code != 0 && !stopping) {  // a signal (crash), or no linger: stop at once
        stopping = true;
        t_stop = std::chrono::steady_clock::now();
        signal_all(SIGTERM);
      }
      continue;
    }
    if (lingering && !stopping && since(t_linger) > linger) {
      stopping = true;
      t_stop = std::chrono::steady_clock::now();
      signal_all(SIGTERM);
    }
    if (g_signal && !stopping) {  // forwarded; the ranks' exits decide the status
      stopping = true;
      t_stop = std::chrono::steady_clock::now();
      signal_all(g_signal);
      if (rc == 0) rc = 128 + g_signal;
    }
    if (stopping && since(t_stop) > grace) signal_all(SIGKILL);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  return rc;
}
