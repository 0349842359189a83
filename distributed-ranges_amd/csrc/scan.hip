// scan.hip -- single-pass inclusive scan (decoupled look-back) for gfx950.
//
// Replaces phases 1 and 3 of shp::inclusive_scan
// (include/dr/shp/algorithms/inclusive_scan.hpp:176-227: oneDPL
// inclusive_scan_async per zipped piece + single_task copy of the piece's
// last value; :244-265: a SECOND full pass x = op(x, carry) with
// oneDPL for_each_async).  Here the carry is folded in-flight: one read
// and one write per element (8 B/elem for 4-byte types) instead of ~16.
//
// Tile = 256 threads x 4 vectors x 16 B (4096 f32/i32, 2048 f64/i64).
//   1. tile index from an atomic counter (dispatch order is not a contract
//      on gfx950, so tiles are numbered in the order blocks START; every
//      predecessor of a tile is then already running -> forward progress);
//   2. 4 independent 16-byte loads per thread (1 KiB per wave-instruction);
//   3. per-vector serial scan, 4 interleaved wave scans (shfl_up), wave
//      totals through LDS -> tile aggregate;
//   4. wave 0 publishes the aggregate and looks back over 64 predecessor
//      tiles per step (one flag per lane, ballot, wave reduce), then
//      publishes its inclusive prefix;
//   5. every element: out = excl (ACC) op local (fp32 in-tile for f32,
//      fp64 inter-tile carries: SURVEY.md 8d tolerance analysis).
// Inter-workgroup hand-off follows MI355X_MICROARCH "Valid forms" row 1:
// payload and flag are agent-scope relaxed atomics (sc1), the producer lane
// drains vmcnt between payload and flag, the consumer polls the flag and
// only then loads the payload (sc1).  Flags are zeroed by a memset node
// before every launch; every spin is bounded and reports through the
// segment's error word.
#include "common.hpp"

#include <type_traits>

namespace drhip {

constexpr int kScanThreads = 256;
constexpr int kScanWaves = kScanThreads / kWave;
constexpr int kScanU = 4;
constexpr unsigned kSpinLimit = 1u << 24;

template <int OP, typename T>
using scan_acc_t = std::conditional_t<std::is_floating_point_v<T>, double,
                                      typename compute_of<OP, T>::type>;

enum : unsigned { FLAG_NONE = 0, FLAG_AGG = 1, FLAG_INCL = 2 };

struct ScanState {
  unsigned *counter;
  unsigned *flags;
  uint64_t *agg;
  uint64_t *incl;
};

template <typename A> struct ScanArgs {
  int has_carry;
  A carry;
  const A *carry_dev;
  A *total;
  unsigned *err;
};

__device__ __forceinline__ void store_relaxed(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_flag(unsigned *p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned load_flag(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_relaxed(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publish value then flag from ONE lane, with the payload drained first.
__device__ __forceinline__ void publish(uint64_t *slot, uint64_t bits, unsigned *flag, unsigned f) {
  store_relaxed(slot, bits);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  store_flag(flag, f);
}

// Wave-0 look-back: returns op-fold of every tile before `tile`.
template <int OP, typename A>
__device__ A lookback(const ScanState st, long tile, int lane, unsigned *err) {
  A excl = Op<OP, A>::identity();
  long pred = tile - 1;
  unsigned spins = 0;
  while (true) {
    const long idx = pred - lane;
    const unsigned f = idx >= 0 ? load_flag(st.flags + idx) : (unsigned)FLAG_INCL;
    const uint64_t incl_mask = __ballot(f == FLAG_INCL);
    const uint64_t zero_mask = __ballot(f == FLAG_NONE);
    const int k = incl_mask ? __builtin_ctzll(incl_mask) : kWave;
    const uint64_t before = k == kWave ? ~0ull : ((1ull << k) - 1ull);
    if (zero_mask & before) {
      if (++spins > kSpinLimit) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    A v = Op<OP, A>::identity();
    if (lane < k) v = from_bits64<A>(load_relaxed(st.agg + idx));
    else if (lane == k) v = from_bits64<A>(load_relaxed(st.incl + idx));
    v = wave_reduce<OP>(v);
    excl = Op<OP, A>::apply(v, excl);
    if (k < kWave) break;
    pred -= kWave;
  }
  return excl;
}

template <int OP, typename T, bool ALIGNED>
__global__ __launch_bounds__(kScanThreads) void scan_kernel(const T *in, T *out,
                                                           size_t n, ScanState st, int has_init,
                                                           typename compute_of<OP, T>::type init,
                                                           ScanArgs<scan_acc_t<OP, T>> a) {
  using C = typename compute_of<OP, T>::type;
  using A = scan_acc_t<OP, T>;
  using OpC = Op<OP, C>;
  using OpA = Op<OP, A>;
  constexpr int V = Vec16<T>::N;
  constexpr size_t TILE = (size_t)kScanThreads * kScanU * V;

  __shared__ unsigned s_tile;
  __shared__ C s_wt[kScanU][kScanWaves];
  __shared__ A s_excl;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wid = tid / kWave;

  if (tid == 0) s_tile = atomicAdd(st.counter, 1u);
  __syncthreads();
  const size_t tile = s_tile;
  const size_t ntiles = (n + TILE - 1) / TILE;
  const size_t base = tile * TILE;
  const bool full = base + TILE <= n;

  // ---- load
  C v[kScanU][V];
  if (ALIGNED && full) {
    const Vec16<T> *src = reinterpret_cast<const Vec16<T> *>(in + base);
    Vec16<T> r[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; u++) r[u] = src[u * kScanThreads + tid];
#pragma unroll
    for (int u = 0; u < kScanU; u++)
#pragma unroll
      for (int j = 0; j < V; j++) v[u][j] = (C)r[u].v[j];
  } else {
#pragma unroll
    for (int u = 0; u < kScanU; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        size_t g = base + ((size_t)u * kScanThreads + tid) * V + j;
        v[u][j] = g < n ? (C)in[g] : OpC::identity();
      }
  }
  if (has_init && tile == 0 && tid == 0) v[0][0] = OpC::apply(init, v[0][0]);

  // ---- in-thread scan of each vector
#pragma unroll
  for (int u = 0; u < kScanU; u++)
#pragma unroll
    for (int j = 1; j < V; j++) v[u][j] = OpC::apply(v[u][j - 1], v[u][j]);

  // ---- wave scans of the per-thread totals (4 independent chains)
  C wincl[kScanU];
#pragma unroll
  for (int u = 0; u < kScanU; u++) wincl[u] = v[u][V - 1];
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
#pragma unroll
    for (int u = 0; u < kScanU; u++) {
      C y = shfl_up(wincl[u], d);
      if (lane >= d) wincl[u] = OpC::apply(y, wincl[u]);
    }
  }
  if (lane == kWave - 1) {
#pragma unroll
    for (int u = 0; u < kScanU; u++) s_wt[u][wid] = wincl[u];
  }
  __syncthreads();

  // ---- block prefix of (sub-tile u, wave w) and tile aggregate
  C pre[kScanU];
  C run = OpC::identity();
#pragma unroll
  for (int u = 0; u < kScanU; u++) {
#pragma unroll
    for (int w = 0; w < kScanWaves; w++) {
      if (w == wid) pre[u] = run;
      run = OpC::apply(run, s_wt[u][w]);
    }
  }
  const C agg = run;

  // thread-exclusive prefix within its vector slot
  C tpre[kScanU];
#pragma unroll
  for (int u = 0; u < kScanU; u++) {
    C wex = shfl_up(wincl[u], 1);
    tpre[u] = lane == 0 ? pre[u] : OpC::apply(pre[u], wex);
  }

  // ---- publish + look-back (wave 0)
  if (wid == 0) {
    A excl;
    if (tile == 0) {
      excl = OpA::identity();
      if (a.has_carry) excl = a.carry;
      if (a.carry_dev) excl = OpA::apply(excl, *a.carry_dev);
      if (lane == 0) publish(st.incl, to_bits64(OpA::apply(excl, (A)agg)), st.flags, FLAG_INCL);
    } else {
      if (lane == 0) publish(st.agg + tile, to_bits64((A)agg), st.flags + tile, FLAG_AGG);
      excl = lookback<OP, A>(st, (long)tile, lane, a.err);
      if (lane == 0) publish(st.incl + tile, to_bits64(OpA::apply(excl, (A)agg)), st.flags + tile, FLAG_INCL);
    }
    if (lane == 0) {
      s_excl = excl;
      if (tile == ntiles - 1 && a.total) *a.total = OpA::apply(excl, (A)agg);
    }
  }
  __syncthreads();
  const A excl = s_excl;

  // ---- combine and store
  if (ALIGNED && full) {
    Vec16<T> *dst = reinterpret_cast<Vec16<T> *>(out + base);
#pragma unroll
    for (int u = 0; u < kScanU; u++) {
      Vec16<T> r;
#pragma unroll
      for (int j = 0; j < V; j++) r.v[j] = (T)OpA::apply(excl, (A)OpC::apply(tpre[u], v[u][j]));
      dst[u * kScanThreads + tid] = r;
    }
  } else {
#pragma unroll
    for (int u = 0; u < kScanU; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        size_t g = base + ((size_t)u * kScanThreads + tid) * V + j;
        if (g < n) out[g] = (T)OpA::apply(excl, (A)OpC::apply(tpre[u], v[u][j]));
      }
  }
}

template <typename A> __global__ void write_scalar(A *p, A v) { *p = v; }

template <typename T, int OP>
static int launch_scan(Segment *s, int seg, const T *in, T *out, size_t n, const void *init_host,
                       const void *carry_host, const void *carry_dev, void *total) {
  using C = typename compute_of<OP, T>::type;
  using A = scan_acc_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  constexpr size_t TILE = (size_t)kScanThreads * kScanU * V;

  ScanArgs<A> a{};
  a.has_carry = carry_host != nullptr;
  if (carry_host) memcpy(&a.carry, carry_host, sizeof(A));
  a.carry_dev = (const A *)carry_dev;
  a.total = (A *)total;
  a.err = s->err;
  C init = Op<OP, C>::identity();
  if (init_host) {
    T t;
    memcpy(&t, init_host, sizeof(T));
    init = (C)t;
  }
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (n == 0) {
    if (total) {
      if (carry_dev) return set_error(DRHIP_ERR_UNSUPPORTED, "scan: n == 0 with carry_dev");
      A t = a.has_carry ? a.carry : Op<OP, A>::identity();
      if (init_host) t = Op<OP, A>::apply(t, (A)init);
      hipLaunchKernelGGL((write_scalar<A>), dim3(1), dim3(1), 0, s->stream, (A *)total, t);
      DRHIP_CHECK_LAUNCH();
    }
    return DRHIP_OK;
  }
  const size_t ntiles = (n + TILE - 1) / TILE;
  if (ntiles > 0xFFFFFFF0ull) return set_error(DRHIP_ERR_BAD_ARG, "scan: too many tiles");
  const size_t hdr = 256;
  const size_t flags_b = (ntiles * sizeof(unsigned) + 255) & ~size_t(255);
  const size_t vals_b = (ntiles * sizeof(uint64_t) + 255) & ~size_t(255);
  int rc = ensure_workspace(seg, hdr + flags_b + 2 * vals_b);
  if (rc) return rc;
  char *ws = (char *)s->ws;
  ScanState st;
  st.counter = (unsigned *)ws;
  st.flags = (unsigned *)(ws + hdr);
  st.agg = (uint64_t *)(ws + hdr + flags_b);
  st.incl = (uint64_t *)(ws + hdr + flags_b + vals_b);
  // Re-initialise every call: counter + flags (one contiguous block).
  DRHIP_CHECK_HIP(hipMemsetAsync(ws, 0, hdr + flags_b, s->stream));
  const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if (aligned)
    hipLaunchKernelGGL((scan_kernel<OP, T, true>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, st, init_host != nullptr, init, a);
  else
    hipLaunchKernelGGL((scan_kernel<OP, T, false>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, st, init_host != nullptr, init, a);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_inclusive_scan(int seg, int dtype, int op, const void *in, void *out, size_t n,
                                    const void *init_host, const void *carry_host,
                                    const void *carry_dev, void *total_acc) {
  DRHIP_GET_SEG(s, seg);
  if ((!in || !out) && n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan: null pointer");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      return launch_scan<T, OP>(s, seg, (const T *)in, (T *)out, n, init_host, carry_host, carry_dev,
                                total_acc);
    });
  });
}
