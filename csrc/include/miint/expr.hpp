// Runtime integrands: f(x) given as an expression, compiled for gfx950 with hipRTC.
//
// The reference's integrand is hard-wired (riemann.cpp:37 `sin(x)`, cintegrate.cu:68) and
// changing it means editing the source and recompiling (no argv, no config).
// Here `riemann --expr "exp(-x*x)" --a 0 --b 3` (or kernels.riemann_expr in Python) turns
// the expression into a HIP device function `double f(double x) { return (EXPR); }`, builds a
// partial-sum kernel and a finalize kernel around it with hipRTC
// (--offload-arch=gfx950 -O3), loads the code object and integrates:
//
//   miint_expr_partials  2048 x 256 lanes, each a contiguous run of samples walked with an
//                        exact fp64 index, every sample evaluated in fp64 (4 accumulators),
//                        wave64 butterfly (__shfl_xor) + 4-wave LDS sum -> one partial per
//                        workgroup
//   miint_expr_finalize  one workgroup sums the partials in index order -> h * scale * sum
//
// Fixed grid and fixed reduction order: bitwise reproducible. Compiled programs are cached
// per (expression, device) in the process. The expression is one C++ expression over `x`
// using the HIP device math library (sin, exp, pow, ...): statements, braces, `asm` and
// string/char literals are rejected before anything is compiled.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "miint/comm.hpp"
#include "miint/common.hpp"
#include "miint/runtime.hpp"

namespace miint {

// Throws unless `expr` is one C++ expression over x (allowed characters only; no statements,
// braces, literals, asm/volatile/goto or __builtin_amdgcn*). Shared by the GPU and host JITs.
void expr_check(const std::string& expr);
// The kernel source generated for `expr` (throws on a rejected expression).
std::string expr_source(const std::string& expr);
// Compile `expr` for gfx950 with hipRTC (no device needed); returns the code object. Throws
// with the compiler log on failure.
std::string expr_compile(const std::string& expr);

class ExprIntegrator {
 public:
  ExprIntegrator(const std::string& expr, int device, int grid = 2048);
  ~ExprIntegrator();
  ExprIntegrator(const ExprIntegrator&) = delete;
  ExprIntegrator& operator=(const ExprIntegrator&) = delete;
  // h * scale * sum f(a + (i + off) h) over samples [begin, begin + count) of an n-sample
  // rule on [a, b]; with a communicator the ranks' values are all-reduced (every rank gets
  // the global sum). Synchronous.
  double integrate(double a, double b, uint64_t n, Rule rule, uint64_t begin, uint64_t count,
                   double scale = 1.0, const Comm* comm = nullptr);
  // Device ms per integration over `iters` back-to-back integrations (events, no host sync
  // between them), for the same arguments. at_start runs on the host right before the first
  // event is recorded (a multi-rank caller's barrier), at_end right before the last one.
  double time(double a, double b, uint64_t n, Rule rule, uint64_t begin, uint64_t count,
              int iters, const std::function<void()>& at_start = {},
              const std::function<void()>& at_end = {});
  const std::string& expression() const { return expr_; }

 private:
  void enqueue(double a, double h, double off, uint64_t begin, uint64_t count, double scale,
               hipStream_t s);
  std::string expr_;
  int device_, grid_;
  hipModule_t module_ = nullptr;
  hipFunction_t partials_fn_ = nullptr, finalize_fn_ = nullptr;
  Stream stream_;
  DeviceBuffer<double> partials_, out_;
  PinnedBuffer<double> host_;
  Event e0_, e1_;
};

}  // namespace miint
