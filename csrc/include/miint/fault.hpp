// Fault injection for the multi-rank agreement tests (SURVEY §5 "Failure detection": the
// reference checks nothing; these hooks let tests prove that a slow or failing rank shows up
// in rank 0's record and exit status). Off unless the variables are set; each reads its
// environment once.
//
//   MIINT_FAULT_RANK=r            the rank the faults below apply to (default: none)
//   MIINT_FAULT_DELAY_MS=ms       rank r holds its end-of-timing mark back by ms (a slow rank:
//                                 the timed interval of every other rank is unchanged)
//   MIINT_FAULT_SCAN_TIMEOUT=1    rank r's train scan reports a hand-off spin timeout
//   MIINT_FAULT_AR_HOST=1         rank r's check of the all-reduce into pinned memory fails
//                                 (RiemannPlan::check_allreduce_to_host: every rank then
//                                 falls back to the device buffer + copy)
#pragma once

#include <chrono>
#include <cstdlib>
#include <thread>

namespace miint {
namespace fault {

inline int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return (v && *v) ? std::atoi(v) : d;
}

inline bool targets(int rank) {
  static const int r = env_int("MIINT_FAULT_RANK", -1);
  return r >= 0 && r == rank;
}

// Sleep on the faulted rank (host side: placed before an end-of-timing event is recorded or a
// host clock is read).
inline void delay(int rank) {
  static const int ms = env_int("MIINT_FAULT_DELAY_MS", 0);
  if (ms > 0 && targets(rank)) std::this_thread::sleep_for(std::chrono::milliseconds(ms));
}

inline bool scan_timeout(int rank) {
  static const bool on = env_int("MIINT_FAULT_SCAN_TIMEOUT", 0) != 0;
  return on && targets(rank);
}

inline bool allreduce_to_host_fails(int rank) {
  static const bool on = env_int("MIINT_FAULT_AR_HOST", 0) != 0;
  return on && targets(rank);
}

}  // namespace fault
}  // namespace miint
