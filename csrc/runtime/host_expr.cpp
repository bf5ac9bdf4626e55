// Host side of runtime integrands (see miint/host.hpp, HostExpr).
//
// The expression (checked by expr_check, the same rules as the hipRTC path) goes into a small
// C++ translation unit that sums f over a sample range the way host_kernels.inc does —
// exact fp64 index, per-sample evaluation, lane accumulators in blocks, compensated block
// sums — but with scalar libm calls, as the reference's own loop does (riemann.cpp:34-41).
// The system compiler builds it into a shared object (-O3 -march=native -fPIC -shared; no
// fast-math), which is dlopen'ed and run on the HostPool's threads.
#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>

#include "miint/expr.hpp"
#include "miint/host.hpp"

extern char** environ;

namespace miint {

namespace {

using SumFn = double (*)(double a, double h, double off, unsigned long long i0,
                         unsigned long long n);

std::string host_source(const std::string& expr) {
  return R"(#include <cmath>
using namespace std;
static inline double miint_f(double x) { return ()" + expr + R"(); }
// sum over i in [i0, i0 + n) of f(a + (i + off) h): blocks of 4096 samples, 8 accumulators
// per block (independent: the compiler may vectorise what it can without reassociating),
// block sums added with Kahan compensation
extern "C" double miint_host_expr_sum(double a, double h, double off, unsigned long long i0,
                                      unsigned long long n) {
  double total = 0.0, comp = 0.0;
  for (unsigned long long done = 0; done < n;) {
    const unsigned long long m = n - done < 4096ull ? n - done : 4096ull;
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double base = (double)(i0 + done) + off;
    unsigned long long k = 0;
    for (; k + 8 <= m; k += 8)
      for (int l = 0; l < 8; ++l) acc[l] += miint_f(fma(base + (double)(k + l), h, a));
    for (; k < m; ++k) acc[0] += miint_f(fma(base + (double)k, h, a));
    const double s = ((acc[0] + acc[4]) + (acc[2] + acc[6])) + ((acc[1] + acc[5]) + (acc[3] + acc[7]));
    const double y = s - comp, t = total + y;
    comp = (t - total) - y;
    total = t;
    done += m;
  }
  return total;
}
)";
}

std::string host_compiler() {
  if (const char* c = std::getenv("MIINT_HOST_CXX")) return c;
  struct stat st;
  if (::stat("/opt/rocm/llvm/bin/clang++", &st) == 0) return "/opt/rocm/llvm/bin/clang++";
  return "c++";
}

// Run argv[0] with argv as a child and wait; returns its exit status. posix_spawn, no fork
// of this possibly GPU-initialised process image, and no shell in between: the compiler is
// the child itself, its stdout and stderr redirected to `log` by spawn file actions.
int run_child(const std::vector<std::string>& args, const std::string& log) {
  std::vector<char*> argv;
  for (const auto& s : args) argv.push_back(const_cast<char*>(s.c_str()));
  argv.push_back(nullptr);
  posix_spawn_file_actions_t fa;
  if (::posix_spawn_file_actions_init(&fa) != 0) return -1;
  ::posix_spawn_file_actions_addopen(&fa, 1, log.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
  ::posix_spawn_file_actions_adddup2(&fa, 1, 2);
  pid_t pid = 0;
  const int err = ::posix_spawnp(&pid, argv[0], &fa, nullptr, argv.data(), environ);
  ::posix_spawn_file_actions_destroy(&fa);
  if (err != 0) return -1;
  int st = 0;
  if (::waitpid(pid, &st, 0) < 0) return -1;
  return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
}

// Under rocprofv3 every child process inherits the profiler's preloaded library, which
// initialises the GPU before the compiler's own code runs; a compiler that then execs its
// driver stages is the exec-after-GPU-init this pool refuses. Refuse up front, with the
// reason, as cuda_v_mpi_amd/_native.py does for its build.
void check_not_profiled() {
  const char* pre = std::getenv("LD_PRELOAD");
  MIINT_CHECK(!(pre && std::string(pre).find("rocprofiler") != std::string::npos),
              "host expression: cannot run the host compiler under rocprofv3 (its preload "
              "initialises the GPU in the compiler); compile the expression outside the "
              "profiled process first");
}

struct Compiled {
  void* handle = nullptr;
  SumFn fn = nullptr;
};

Compiled compile_host(const std::string& expr) {
  static std::mutex mu;
  static std::map<std::string, Compiled> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(expr);
  if (it != cache.end()) return it->second;
  expr_check(expr);
  const char* tmp = std::getenv("TMPDIR");
  std::string dir = std::string(tmp && *tmp ? tmp : "/tmp") + "/miint_hostexpr_XXXXXX";
  MIINT_CHECK(::mkdtemp(&dir[0]) != nullptr, "host expression: mkdtemp failed");
  const std::string src = dir + "/f.cpp", so = dir + "/f.so", log = dir + "/log.txt";
  {
    std::ofstream f(src);
    f << host_source(expr);
  }
  check_not_profiled();
  const int rc = run_child({host_compiler(), "-std=c++17", "-O3", "-march=native", "-fPIC",
                            "-shared", "-o", so, src}, log);
  auto cleanup = [&] {  // the loaded object stays mapped; the files can go
    std::remove(src.c_str());
    std::remove(so.c_str());
    std::remove(log.c_str());
    ::rmdir(dir.c_str());
  };
  if (rc != 0) {
    std::ifstream l(log);
    const std::string text((std::istreambuf_iterator<char>(l)), std::istreambuf_iterator<char>());
    cleanup();
    fail("host expression '" + expr + "' does not compile (" + host_compiler() + "): " + text,
         __FILE__, __LINE__);
  }
  Compiled c;
  c.handle = ::dlopen(so.c_str(), RTLD_NOW | RTLD_LOCAL);
  const std::string dl_err = c.handle ? "" : ::dlerror();
  cleanup();
  MIINT_CHECK(c.handle != nullptr, "host expression: dlopen: " + dl_err);
  c.fn = reinterpret_cast<SumFn>(::dlsym(c.handle, "miint_host_expr_sum"));
  MIINT_CHECK(c.fn != nullptr, "host expression: symbol missing");
  return cache[expr] = c;
}

}  // namespace

HostExpr::HostExpr(const std::string& expr) : expr_(expr) {
  fn_ = reinterpret_cast<void*>(compile_host(expr).fn);
}

double HostExpr::integrate(double a, double b, uint64_t n, Rule rule, uint64_t begin,
                           uint64_t count, HostPool& pool) const {
  MIINT_CHECK(n >= 1 && begin + count <= n && begin + count >= begin,
              "host expression slice outside [0, n)");
  const SumFn fn = reinterpret_cast<SumFn>(fn_);
  const double h = (b - a) / static_cast<double>(n), off = rule_offset(rule);
  const int T = pool.threads();
  std::vector<double> part(T, 0.0);
  pool.run([&](int t) {
    uint64_t tb = 0, tc = 0;
    rank_slice(count, t, T, &tb, &tc);
    if (tc) part[t] = fn(a, h, off, begin + tb, tc);
  });
  double s = 0.0;
  for (int t = 0; t < T; ++t) s += part[t];  // thread order
  return s * h;
}

}  // namespace miint
