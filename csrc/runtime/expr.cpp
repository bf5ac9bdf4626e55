// Runtime integrands compiled with hipRTC (see miint/expr.hpp).
#include "miint/expr.hpp"

#include <hip/hiprtc.h>

#include <cctype>
#include <map>
#include <mutex>

namespace miint {

namespace {
constexpr int kExprBlock = 256;
}  // namespace

// One C++ expression over x: no statements, blocks, asm or literals that could smuggle them.
void expr_check(const std::string& e) {
  MIINT_CHECK(!e.empty() && e.size() <= 4096, "expression must be 1..4096 characters");
  for (char c : e) {
    const bool ok = std::isalnum(static_cast<unsigned char>(c)) ||
                    std::string(" \t_.+-*/%(),?:<>=!&|^~").find(c) != std::string::npos;
    MIINT_CHECK(ok, std::string("expression: character '") + c + "' not allowed (one C++ "
                    "expression over x: no ; { } [ ] # quotes or backslashes)");
  }
  // digraphs spell the characters refused above: <% %> <: :> %: are { } [ ] #
  for (const char* dg : {"<%", "%>", "<:", ":>", "%:"})
    MIINT_CHECK(e.find(dg) == std::string::npos,
                std::string("expression: digraph '") + dg + "' not allowed (it spells a brace, "
                "bracket or #)");
  // identifiers that are not math: asm / volatile / goto / the preprocessor are out
  std::string word;
  auto bad = [](const std::string& w) {
    return w == "asm" || w == "__asm" || w == "__asm__" || w == "volatile" || w == "goto" ||
           w == "__builtin_amdgcn_s_sendmsg" || w.rfind("__builtin_amdgcn", 0) == 0;
  };
  for (size_t i = 0; i <= e.size(); ++i) {
    const char c = i < e.size() ? e[i] : ' ';
    if (std::isalnum(static_cast<unsigned char>(c)) || c == '_') {
      word += c;
    } else {
      MIINT_CHECK(!bad(word), "expression: '" + word + "' is not allowed");
      word.clear();
    }
  }
}

namespace {
std::string rtc_error(hiprtcResult r) { return hiprtcGetErrorString(r); }
}  // namespace

std::string expr_source(const std::string& expr) {
  expr_check(expr);
  // hipRTC compiles this with its own HIP headers (device math, __shfl_xor, blockIdx, ...).
  return R"(
__device__ __forceinline__ double miint_f(double x) { return ()" + expr + R"(); }

// Every sample on its own. Lane g owns a contiguous run of the slice (balanced: the first
// n mod lanes lanes take one more) and walks it with an exact fp64 index (idx += 1, exact
// below 2^52), so a sample costs fma(idx, h, a), f and an add: no per-sample 64-bit integer
// to fp64 conversion. Four independent accumulators for ILP.
extern "C" __global__ __launch_bounds__(256) void miint_expr_partials(
    double a, double h, double off, unsigned long long i0, unsigned long long n,
    double* partials) {
  __shared__ double red[4];
  const unsigned long long lanes = (unsigned long long)gridDim.x * 256ull;
  const unsigned long long g = (unsigned long long)blockIdx.x * 256ull + threadIdx.x;
  const unsigned long long q = n / lanes, r = n % lanes;
  const unsigned long long start = g * q + (g < r ? g : r);
  const unsigned cnt = (unsigned)(q + (g < r ? 1ull : 0ull));
  double idx = (double)(i0 + start) + off;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  unsigned k = 0;
  for (; k + 4 <= cnt; k += 4) {
    a0 += miint_f(fma(idx, h, a));
    a1 += miint_f(fma(idx + 1.0, h, a));
    a2 += miint_f(fma(idx + 2.0, h, a));
    a3 += miint_f(fma(idx + 3.0, h, a));
    idx += 4.0;
  }
  for (; k < cnt; ++k) {
    a0 += miint_f(fma(idx, h, a));
    idx += 1.0;
  }
  double acc = (a0 + a1) + (a2 + a3);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);  // wave64 butterfly
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// One workgroup: thread t sums partials t, t + 256, ... in order; fixed-order tree after.
extern "C" __global__ __launch_bounds__(256) void miint_expr_finalize(
    const double* partials, int n, double scale, double* out) {
  __shared__ double red[4];
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) v += partials[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
}
)";
}

std::string expr_compile(const std::string& expr) {
  static std::mutex mu;
  static std::map<std::string, std::string> cache;  // expression -> code object
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(expr);
  if (it != cache.end()) return it->second;
  const std::string src = expr_source(expr);
  hiprtcProgram prog = nullptr;
  hiprtcResult r = hiprtcCreateProgram(&prog, src.c_str(), "miint_expr.hip", 0, nullptr, nullptr);
  MIINT_CHECK(r == HIPRTC_SUCCESS, "hiprtcCreateProgram: " + rtc_error(r));
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  r = hiprtcCompileProgram(prog, 3, opts);
  size_t log_n = 0;
  hiprtcGetProgramLogSize(prog, &log_n);
  std::string log(log_n, '\0');
  if (log_n) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    fail("expression '" + expr + "' does not compile: " + log, __FILE__, __LINE__);
  }
  size_t code_n = 0;
  MIINT_CHECK(hiprtcGetCodeSize(prog, &code_n) == HIPRTC_SUCCESS && code_n > 0,
              "hiprtcGetCodeSize");
  std::string code(code_n, '\0');
  MIINT_CHECK(hiprtcGetCode(prog, &code[0]) == HIPRTC_SUCCESS, "hiprtcGetCode");
  hiprtcDestroyProgram(&prog);
  return cache[expr] = code;
}

ExprIntegrator::ExprIntegrator(const std::string& expr, int device, int grid)
    : expr_(expr), device_(device), grid_(grid), stream_((set_device(device), Stream())) {
  MIINT_CHECK(grid >= 1 && grid <= 65535, "expression grid out of range");
  const std::string code = expr_compile(expr);
  DeviceGuard g(device);
  MIINT_HIP(hipModuleLoadData(&module_, code.data()));
  MIINT_HIP(hipModuleGetFunction(&partials_fn_, module_, "miint_expr_partials"));
  MIINT_HIP(hipModuleGetFunction(&finalize_fn_, module_, "miint_expr_finalize"));
  partials_ = DeviceBuffer<double>(static_cast<size_t>(grid));
  out_ = DeviceBuffer<double>(1);
  host_ = PinnedBuffer<double>(1);
}

ExprIntegrator::~ExprIntegrator() {
  if (module_) {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(stream_.get());
    (void)hipModuleUnload(module_);
  }
}

void ExprIntegrator::enqueue(double a, double h, double off, uint64_t begin, uint64_t count,
                             double scale, hipStream_t s) {
  unsigned long long i0 = begin, n = count;
  double* parts = partials_.get();
  void* args[] = {&a, &h, &off, &i0, &n, &parts};
  MIINT_HIP(hipModuleLaunchKernel(partials_fn_, grid_, 1, 1, kExprBlock, 1, 1, 0, s, args,
                                  nullptr));
  int nb = grid_;
  double sc = scale;
  double* out = out_.get();
  void* fargs[] = {&parts, &nb, &sc, &out};
  MIINT_HIP(hipModuleLaunchKernel(finalize_fn_, 1, 1, 1, kExprBlock, 1, 1, 0, s, fargs,
                                  nullptr));
}

double ExprIntegrator::integrate(double a, double b, uint64_t n, Rule rule, uint64_t begin,
                                 uint64_t count, double scale, const Comm* comm) {
  MIINT_CHECK(n >= 1 && begin + count <= n, "expression slice outside [0, n)");
  DeviceGuard g(device_);
  const double h = (b - a) / static_cast<double>(n);
  hipStream_t s = stream_.get();
  enqueue(a, h, rule_offset(rule), begin, count, h * scale, s);
  if (comm && comm->world() > 1) comm->allreduce_sum(out_.get(), out_.get(), 1, s);
  MIINT_HIP(hipMemcpyAsync(host_.get(), out_.get(), sizeof(double), hipMemcpyDeviceToHost, s));
  stream_.sync();
  return host_[0];
}

double ExprIntegrator::time(double a, double b, uint64_t n, Rule rule, uint64_t begin,
                            uint64_t count, int iters, const std::function<void()>& at_start,
                            const std::function<void()>& at_end) {
  MIINT_CHECK(iters >= 1 && n >= 1 && begin + count <= n, "bad expression timing request");
  DeviceGuard g(device_);
  const double h = (b - a) / static_cast<double>(n);
  hipStream_t s = stream_.get();
  enqueue(a, h, rule_offset(rule), begin, count, h, s);  // warm
  stream_.sync();
  if (at_start) at_start();
  e0_.record(s);
  for (int i = 0; i < iters; ++i) enqueue(a, h, rule_offset(rule), begin, count, h, s);
  if (at_end) at_end();
  e1_.record(s);
  stream_.sync();
  return Event::elapsed_ms(e0_, e1_) / iters;
}

}  // namespace miint
