// roctx tracing (lazy dlopen) and the stream/collective watchdog (see miint/trace.hpp).
#include "miint/trace.hpp"

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <thread>

#include "miint/comm.hpp"
#include "miint/common.hpp"
#include "miint/runtime.hpp"

namespace miint {

namespace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  bool loaded = false;
};

std::atomic<int> g_enabled{-1};  // -1: read MIINT_ROCTX on first use
std::once_flag g_load_once;
Roctx g_roctx;

void load_roctx() {
  std::call_once(g_load_once, [] {
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "libroctx64.so.4", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      g_roctx.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      g_roctx.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      g_roctx.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
      if (g_roctx.push && g_roctx.pop) {
        g_roctx.loaded = true;
        return;
      }
    }
  });
}

}  // namespace

namespace {
void crash_handler(int sig) {
  static const char msg[] = "\nmiint: fatal signal, native backtrace:\n";
  (void)!::write(2, msg, sizeof(msg) - 1);
  void* frames[64];
  const int n = ::backtrace(frames, 64);
  ::backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}
}  // namespace

void install_crash_handler_from_env() {
  const char* v = std::getenv("MIINT_CRASH_TRACE");
  if (!v || v[0] != '1') return;
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT}) ::signal(sig, crash_handler);
}

void enable_tracing(bool on) {
  g_enabled = on ? 1 : 0;
  if (on) load_roctx();
}

bool tracing_enabled() {
  int e = g_enabled.load(std::memory_order_relaxed);
  if (e < 0) {
    const char* v = std::getenv("MIINT_ROCTX");
    enable_tracing(v && v[0] == '1');
    e = g_enabled.load();
  }
  return e == 1 && g_roctx.loaded;
}

void trace_push(const char* name) {
  if (g_roctx.push) g_roctx.push(name);
}
void trace_pop() {
  if (g_roctx.pop) g_roctx.pop();
}
void trace_mark(const char* name) {
  if (tracing_enabled() && g_roctx.mark) g_roctx.mark(name);
}

double wait_with_timeout(hipStream_t s, double timeout_s, const Comm* comm) {
  const double t0 = wall_seconds();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return wall_seconds() - t0;
    if (q != hipErrorNotReady) MIINT_HIP(q);
    if (comm) comm->check_async();  // throws on an RCCL async error (e.g. a dead peer)
    const double waited = wall_seconds() - t0;
    if (waited > timeout_s) {
      if (comm) comm->abort();
      fail("stream did not drain within " + std::to_string(timeout_s) +
               " s (collective hang or runaway kernel); communicator aborted",
           __FILE__, __LINE__);
    }
    // Poll tightly while a drain is plausible: the caller times right after this returns
    // (bench.py brackets its K steps with it on every multi-GPU run), and 1 ms sleeps added
    // up to 1 ms per timed region (2.5 us per step over 400 steps). Back off after 2 s.
    if (waited < 2.0)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

}  // namespace miint
