// Single-pass decoupled look-back inclusive scan (fp64) for gfx950.
//
// Replaces 4main.c's distributed prefix scan (SURVEY P4, 4main.c:95-221): local serial scan
// per rank, MPI_Send of every slice to root, an O(T) *serial* carry loop on root
// (4main.c:152-153) and a 144 MB MPI_Bcast. On one GPU the whole 18 M-element recurrence
// is one launch: each workgroup scans a 4096-element tile in registers/LDS (DPP wave scan
// + LDS across waves), publishes its aggregate, and obtains its exclusive prefix by a
// wave-parallel look-back over up to 64 predecessors at a time. Across GPUs the only
// traffic is an allgather of one fp64 total per rank (csrc/runtime/trainscan.cpp).
//
// Inter-workgroup protocol: the write-once slots of handoff.hpp. Per tile there are two
// slots, its aggregate and its inclusive prefix, each filled with the unset pattern by the
// launcher's memset and written ONCE per launch with a relaxed agent-scope atomic store; a
// look-back lane polls its predecessor's prefix slot, then its aggregate slot, and the value
// it reads is the status — no separate flag whose ordering against the value the memory
// model would have to guarantee. Tile ids come from an atomic counter so a tile only ever
// waits on tiles that are already running (forward progress under any dispatch order).
// Bounded spins: a predecessor that never publishes makes the prefix NaN (every later
// output poisoned) and raises the timeout word, which every host path turns into an error.
#include <hip/hip_runtime.h>

#include "miint/common.hpp"
#include "miint/handoff.hpp"
#include "miint/kernels.hpp"
#include "miint/trainscan.hpp"
#include "miint/wave_reduce.hpp"

namespace miint {
namespace {

constexpr int kB = 256;
constexpr int kItems = 16;                 // per thread
constexpr int kTileN = kB * kItems;        // 4096 elements = 32 KB per tile
struct ScanState {
  unsigned* counter;   // dynamic tile id
  double* agg;         // per tile aggregate (write-once slot)
  double* pref;        // per tile inclusive prefix (write-once slot)
  unsigned* timeout;   // set if any spin gave up (every host path turns it into an error)
};

// Wave 0: exclusive prefix of `tile` by look-back (lanes examine tile-1-lane).
__device__ double look_back(ScanState st, unsigned tile) {
  const int lane = threadIdx.x & 63;
  double excl = 0.0;
  long base = static_cast<long>(tile) - 1;
  for (;;) {
    const long j = base - lane;
    bool is_pref = true;  // lanes past the front act as "prefix 0"
    double v = 0.0;
    if (j >= 0) {
      unsigned spins = 0;
      for (;;) {
        v = slot_load(st.pref + j);
        if (!slot_unset(v)) break;
        v = slot_load(st.agg + j);
        if (!slot_unset(v)) {
          is_pref = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSlotSpinLimit) {
          __hip_atomic_store(st.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = __builtin_nan("");
          break;
        }
      }
    }
    // first lane (closest predecessor) holding an inclusive prefix
    const unsigned long long pm = __ballot(is_pref);
    const int stop = pm ? __builtin_ctzll(pm) : 64;
    const double mine = lane <= stop ? v : 0.0;
    excl += wave_sum(mine);
    if (pm) break;
    base -= 64;
  }
  return excl;
}

// Load/store a tile in the "striped" order (coalesced 8-B per lane) through LDS and hand
// each thread kItems consecutive elements ("blocked" order) for the serial part.
template <class Load>
__device__ __forceinline__ void scan_tile(ScanState st, uint64_t n, double* out,
                                          const double* carry_in, Load load) {
  __shared__ double buf[kTileN + kTileN / 32];  // +1 pad per 32 to break bank conflicts
  __shared__ double red[kB / kWave];
  __shared__ unsigned tile_sh;
  __shared__ double prefix_sh;
  if (threadIdx.x == 0)
    tile_sh = __hip_atomic_fetch_add(st.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned tile = tile_sh;
  const uint64_t t0 = static_cast<uint64_t>(tile) * kTileN;
  auto pad = [](int i) { return i + (i >> 5); };
  // striped load
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int i = k * kB + threadIdx.x;
    const uint64_t g = t0 + i;
    buf[pad(i)] = g < n ? load(g) : 0.0;
  }
  __syncthreads();
  // blocked serial scan
  double v[kItems];
  double run = 0.0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    run += buf[pad(threadIdx.x * kItems + k)];
    v[k] = run;
  }
  double total;
  const double incl = block_inclusive_scan<kB>(run, red, &total);
  const double thread_excl = incl - run;
  // look-back for the tile's exclusive prefix (wave 0), published ASAP
  if (threadIdx.x < 64) {
    double excl = 0.0;
    if (tile == 0) {
      if (threadIdx.x == 0) slot_store(st.pref + tile, total);
    } else {
      if (threadIdx.x == 0) slot_store(st.agg + tile, total);
      excl = look_back(st, tile);
      if (threadIdx.x == 0) slot_store(st.pref + tile, excl + total);
    }
    if (threadIdx.x == 0) prefix_sh = excl + (carry_in ? carry_in[0] : 0.0);
  }
  __syncthreads();
  const double add = prefix_sh + thread_excl;
#pragma unroll
  for (int k = 0; k < kItems; ++k) buf[pad(threadIdx.x * kItems + k)] = v[k] + add;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int i = k * kB + threadIdx.x;
    const uint64_t g = t0 + i;
    if (g < n) out[g] = buf[pad(i)];
  }
}

__global__ __launch_bounds__(kB) void scan_kernel(const double* in, double* out, uint64_t n,
                                                  ScanState st, const double* carry_in) {
  scan_tile(st, n, out, carry_in, [&](uint64_t g) { return in[g]; });
}

constexpr int kMaxTable = 2048;

__global__ __launch_bounds__(kB) void interp_scan_kernel(const double* table, int table_n,
                                                         double dt, uint64_t i0, uint64_t n,
                                                         uint64_t win_lo, uint64_t win_hi,
                                                         double* out, ScanState st,
                                                         const double* carry_in) {
  __shared__ double tab[kMaxTable];
  for (int k = threadIdx.x; k < table_n; k += kB) tab[k] = table[k];
  __syncthreads();
  const int nseg = table_n - 1;
  scan_tile(st, n, out, carry_in, [&](uint64_t g) {
    const uint64_t i = i0 + g;
    if (i < win_lo || i >= win_hi) return 0.0;  // parity emulation of per-rank fill windows
    const double t = dt * static_cast<double>(i);
    int s = static_cast<int>(t);
    s = s < 0 ? 0 : (s >= nseg ? nseg - 1 : s);
    const double v0 = tab[s];
    return fma(tab[s + 1] - v0, t - static_cast<double>(s), v0);
  });
}

__global__ __launch_bounds__(kB) void add_carry_kernel(double* x, uint64_t n, const double* c) {
  const double cv = c[0];
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * kB;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kB + threadIdx.x; i < n; i += lanes)
    x[i] += cv;
}

__global__ void exclusive_carry_kernel(const double* totals, int rank, double* out) {
  double c = 0.0;
  for (int q = 0; q < rank; ++q) c += totals[q];  // fixed order: identical on every rank
  out[0] = c;
}

// State: {counter, timeout} (16 B, zeroed per launch), then the agg and pref slots (filled
// with the unset pattern per launch).
ScanState carve(void* state, uint64_t ntiles) {
  char* p = static_cast<char*>(state);
  ScanState st;
  st.counter = reinterpret_cast<unsigned*>(p);
  st.timeout = reinterpret_cast<unsigned*>(p + 4);
  st.agg = reinterpret_cast<double*>(p + 16);
  st.pref = st.agg + ntiles;
  return st;
}

void arm_state(void* state, uint64_t ntiles, hipStream_t stream) {
  MIINT_HIP(hipMemsetAsync(state, 0, 16, stream));
  fill_unset_slots(reinterpret_cast<double*>(static_cast<char*>(state) + 16), 2 * ntiles, stream);
}

}  // namespace

size_t scan_state_bytes(uint64_t n) {
  const uint64_t nt = (n + kTileN - 1) / kTileN;
  return 16 + 2 * nt * sizeof(double);
}

void launch_inclusive_scan(const double* in, double* out, uint64_t n, void* state,
                           const double* carry_in, hipStream_t stream) {
  MIINT_CHECK(n >= 1, "empty scan");
  const uint64_t nt = (n + kTileN - 1) / kTileN;
  MIINT_CHECK(nt < (1u << 31), "scan too large");
  ScanState st = carve(state, nt);
  arm_state(state, nt, stream);
  scan_kernel<<<static_cast<unsigned>(nt), kB, 0, stream>>>(in, out, n, st, carry_in);
  MIINT_HIP(hipGetLastError());
}

void launch_interp_scan(const double* table, int table_n, double dt, uint64_t i0, uint64_t n,
                        double* out, void* state, const double* carry_in, hipStream_t stream) {
  launch_interp_scan_window(table, table_n, dt, i0, n, 0, ~uint64_t(0), out, state, carry_in,
                            stream);
}

void launch_interp_scan_window(const double* table, int table_n, double dt, uint64_t i0,
                               uint64_t n, uint64_t win_lo, uint64_t win_hi, double* out,
                               void* state, const double* carry_in, hipStream_t stream) {
  MIINT_CHECK(n >= 1, "empty scan");
  MIINT_CHECK(table_n >= 2 && table_n <= kMaxTable, "table size must be in [2, 2048]");
  const uint64_t nt = (n + kTileN - 1) / kTileN;
  ScanState st = carve(state, nt);
  arm_state(state, nt, stream);
  interp_scan_kernel<<<static_cast<unsigned>(nt), kB, 0, stream>>>(
      table, table_n, dt, i0, n, win_lo, win_hi, out, st, carry_in);
  MIINT_HIP(hipGetLastError());
}

void launch_add_carry(double* x, uint64_t n, const double* carry, hipStream_t stream) {
  if (n == 0) return;
  const int grid = static_cast<int>(std::min<uint64_t>((n + kB - 1) / kB, 4096));
  add_carry_kernel<<<grid, kB, 0, stream>>>(x, n, carry);
  MIINT_HIP(hipGetLastError());
}

void launch_exclusive_carry(const double* totals, int rank, double* out, hipStream_t s) {
  exclusive_carry_kernel<<<1, 1, 0, s>>>(totals, rank, out);
  MIINT_HIP(hipGetLastError());
}

unsigned scan_timeout_flag(const void* state, hipStream_t stream) {
  unsigned v = 0;
  MIINT_HIP(hipMemcpyAsync(&v, static_cast<const char*>(state) + 4, sizeof(unsigned),
                           hipMemcpyDeviceToHost, stream));
  MIINT_HIP(hipStreamSynchronize(stream));
  return v;
}

}  // namespace miint
