// Loopback-transport kernel: the element-wise sum behind LoopbackComm's all-reduce / reduce
// (see miint/comm.hpp). W logical ranks live on one device, so "the network" is a read of
// every rank's send buffer; the sum runs in fixed rank order (q = 0 .. W-1), making the
// result independent of which rank's stream issues it and bitwise reproducible.
//
// Purely bandwidth-bound and tiny in practice (a bucket of step results, a few scalars):
// a grid-stride loop with one fp64 per lane per iteration is all it needs.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "miint/comm.hpp"

namespace miint {
namespace {

__global__ __launch_bounds__(256) void loopback_sum_kernel(LoopbackPtrs src, int w, size_t count,
                                                           double* out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
       i += stride) {
    double acc = src.p[0][i];
    for (int q = 1; q < w; ++q) acc += src.p[q][i];
    out[i] = acc;
  }
}

}  // namespace

void launch_loopback_sum(const LoopbackPtrs& src, int w, size_t count, double* out,
                         hipStream_t s) {
  MIINT_CHECK(w >= 1 && w <= kMaxLoopbackRanks, "loopback sum: bad rank count");
  for (int q = 0; q < w; ++q) MIINT_CHECK(src.p[q] != nullptr, "loopback sum: null send buffer");
  if (count == 0) return;
  const size_t blocks = std::min<size_t>((count + 255) / 256, 2048);
  loopback_sum_kernel<<<static_cast<unsigned>(blocks), 256, 0, s>>>(src, w, count, out);
  MIINT_HIP(hipGetLastError());
}

}  // namespace miint
