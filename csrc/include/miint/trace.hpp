// Tracing and failure detection.
//
// The reference's only instrumentation is a wall clock around the whole program
// (clock_gettime in cintegrate.cu:104,139 / riemann.cpp:51,91 / 4main.c:67,238)
// and it checks no error codes at all (B8). Here:
//   * roctx ranges around every runtime phase (plan build, graph capture, step batches,
//     collectives), visible in `rocprofv3 --marker-trace`. The roctx library is loaded
//     lazily with dlopen when MIINT_ROCTX=1 (or enable_tracing(true)), so nothing is linked
//     and tracing costs one branch when off;
//   * a collective watchdog: wait_with_timeout() polls a stream and the communicator's
//     asynchronous error state, aborts the communicator and throws on timeout or error
//     (a dead peer no longer hangs every other rank forever).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace miint {

class Comm;

void enable_tracing(bool on);
bool tracing_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

// Failure detection for native crashes: with MIINT_CRASH_TRACE=1 a SIGSEGV/SIGBUS/SIGABRT
// handler writes the native backtrace (glibc backtrace_symbols_fd) to stderr before the
// default action runs. Installed by the Python module and the CLIs at start-up.
void install_crash_handler_from_env();

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(tracing_enabled()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

// Wait for `s` to drain; if `comm` reports an asynchronous error or `timeout_s` passes,
// abort the communicator (if any) and throw miint::Error. Returns seconds waited.
double wait_with_timeout(hipStream_t s, double timeout_s, const Comm* comm = nullptr);

}  // namespace miint
