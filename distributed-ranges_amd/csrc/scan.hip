// scan.hip -- launcher + C-ABI entry of the single-pass inclusive scan
// (kernel: scan_kernel.hpp).
#include "scan_kernel.hpp"

#include <algorithm>

namespace drhip {

template <typename A> __global__ void write_scalar(A *p, A v) { *p = v; }

// *res = parts[0] op ... op parts[w-1], left to right (the order the scan
// kernels fold the gathered partials in): an empty segment's scan still
// delivers the reduce result of the ranks that hold elements
template <int OP, typename A> __global__ void fold_parts_kernel(const A *parts, int w, A *res) {
  A acc = parts[0];
  for (int k = 1; k < w; k++) acc = Op<OP, A>::apply(acc, parts[k]);
  *res = acc;
}

template <int OP, typename A> static int launch_fold_parts(Segment *s, const void *parts, int w, void *res) {
  hipLaunchKernelGGL((fold_parts_kernel<OP, A>), dim3(1), dim3(1), 0, s->stream, (const A *)parts, w, (A *)res);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

struct Gathered {
  const void *parts = nullptr; // w ACC values (drhip_allgather's output)
  int w = 0, rank = 0;
  void *result = nullptr;
};

template <typename T, int OP, int UB>
static int launch_scan(Segment *s, int seg, const T *in, T *out, size_t n, const void *init_host,
                       const void *carry_host, const void *carry_dev, void *total, const Gathered &g = {}) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  constexpr int U = scan_u<T, C, UB>();
  constexpr size_t TILE = (size_t)kScanThreads * U * V;

  ScanArgs<A> a{};
  a.has_carry = carry_host != nullptr;
  if (carry_host) memcpy(&a.carry, carry_host, sizeof(A));
  a.carry_dev = (const A *)carry_dev;
  a.parts = (const A *)g.parts;
  a.parts_w = g.w;
  a.parts_rank = g.rank;
  a.fold_res = (A *)g.result;
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
      if (carry_dev || g.parts) return set_error(DRHIP_ERR_UNSUPPORTED, "scan: n == 0 with a device carry");
      A t = a.has_carry ? a.carry : Op<OP, A>::identity();
      if (init_host) t = Op<OP, A>::apply(t, (A)init);
      hipLaunchKernelGGL((write_scalar<A>), dim3(1), dim3(1), 0, s->stream, (A *)total, t);
      DRHIP_CHECK_LAUNCH();
    }
    if (g.parts && g.result) return launch_fold_parts<OP, A>(s, g.parts, g.w, g.result);
    return DRHIP_OK;
  }
  const size_t ntiles = (n + TILE - 1) / TILE;
  constexpr size_t GB = granule_bytes<OP, T>();
  if (ntiles * GB > 0x7FFFFFF0ull) return set_error(DRHIP_ERR_BAD_ARG, "scan: too many tiles");
  const size_t hdr = 256;
  const size_t gran_b = (ntiles * GB + 1023) & ~size_t(1023); // quarters of whole 256-B blocks
  int rc = ensure_workspace(seg, hdr + gran_b);
  if (rc) return rc;
  char *ws = (char *)s->ws;
  granules_t<OP, T> gr;
  gr.base = ws + hdr;
  gr.bytes = (int)gran_b;
  // Re-initialise every call: tile counter + granules (one contiguous block).
  DRHIP_CHECK_HIP(hipMemsetAsync(ws, 0, hdr + gran_b, s->stream));
  const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if (aligned)
    hipLaunchKernelGGL((scan_kernel<OP, T, true, U>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, (unsigned *)ws, gr, init_host != nullptr, init, a);
  else
    hipLaunchKernelGGL((scan_kernel<OP, T, false, U>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, (unsigned *)ws, gr, init_host != nullptr, init, a);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

// Tile size by input size: large inputs take twice the bytes per tile (and
// per look-back wait).  The choice is made here, once, so no launcher calls
// another instantiation of itself: a round-3 measurement build with
// DRHIP_SCAN_UBIG == kScanU made the old self-dispatching launcher recurse
// into its own instantiation (infinite recursion, undefined behaviour, a GPU
// fault); tests/test_knob_builds.py compiles the knob values.
template <typename T, int OP>
static int scan_dispatch(Segment *s, int seg, const T *in, T *out, size_t n, const void *init_host,
                         const void *carry_host, const void *carry_dev, void *total, const Gathered &g = {}) {
  if (n * sizeof(T) >= kScanBigBytes)
    return launch_scan<T, OP, kScanUBig>(s, seg, in, out, n, init_host, carry_host, carry_dev, total, g);
  return launch_scan<T, OP, kScanU>(s, seg, in, out, n, init_host, carry_host, carry_dev, total, g);
}

// ------------------------------------------------------------------------
// Reduce + scan over the SAME range (the C2 step): drhip_reduce_tiles reads
// the range once in the scan's own tiles and leaves every tile part's
// exclusive prefix behind, so the scan that follows
// (drhip_inclusive_scan_tiles, scan_wave_given_kernel) needs no look-back,
// LDS or barrier.  The reduce stays 4 B/elem, the scan 8 B/elem.
//
// Tile = kTilesNW wave PARTS; wave w of a block reads part w (contiguous) in
// both kernels.  Layout of the segment's tile buffer (A = the scan's ACC):
//   local[ntiles * kTilesNW]  exclusive prefix of part (t, w) among its
//                             reduce block's tiles
//   block[grid]    exclusive prefix of reduce block b (written by the last
//                  block to finish)
//   bpart[grid]    block totals (`sc1` stores, folded by the last block)
// Reduce block b owns the contiguous tiles [b*per, min((b+1)*per, ntiles)).
// Tile shape (vectors per thread, as kScanU): 2^26..2^30 f32 (reduce + scan
// ms, tools/scan_tiles_ab.py, profiles/r04_scan_tiles_wave_ab.txt): 2 vectors
// per thread in dispatch order 0.128 / 0.255 / 0.511 / 1.034 / 2.043; 32
// claimed in start order 0.145 / 0.274 / 0.526 / 1.027 / 2.015 -- so 2 below
// 2 GiB of input and 32 from there.  Block-level forms measured before it
// and removed (profiles/r04_scan_tiles_ab.txt): one-shot U = 32 / 16 / 8
// 1.41 / 1.425 / 1.665 ms of scan at 2^30, a two-tile pipeline at U = 16
// 1.402.
#ifndef DRHIP_TILES_UBIG
#define DRHIP_TILES_UBIG 32
#endif
#ifndef DRHIP_TILES_U
#define DRHIP_TILES_U 2
#endif
constexpr int kTilesUBig = DRHIP_TILES_UBIG, kTilesU = DRHIP_TILES_U;
constexpr size_t kTilesBigBytes = size_t(1) << 31;
constexpr int kTilesNW = kScanThreads / kWave; // wave parts per tile
constexpr int kRtMaxGrid = 4096;
#ifndef DRHIP_RT_BLOCKS_PER_CU
#define DRHIP_RT_BLOCKS_PER_CU 2
#endif
// reduce_tiles grid: blocks per CU.  2^26 / 2^27 / 2^28 / 2^30 f32
// (tools/scan_tiles_ab.py, profiles/r04_reduce_tiles_grid_ab.txt): 8 per CU
// 0.048 / 0.090 / 0.177 / 0.636 ms, 4 0.044 / 0.086 / 0.169 / 0.636, 2 0.043
// / 0.0835 / 0.166 / 0.635, 16 0.052 / 0.092 / 0.174 / 0.642: fewer, longer
// blocks leave the last block fewer partials to fold
constexpr int kRtBlocksPerCU = DRHIP_RT_BLOCKS_PER_CU;
constexpr int kRtChunk = kWave; // tiles per wave-0 prefix step
// the scan's tile counter: past the reduce's two-level counters
// (done[(1 + g) * 32], g < kRtMaxGrid / 32) inside the kSyncTiles words
constexpr int kRtScanCounter = (kRtMaxGrid / 32 + 2) * 32;
static_assert(kRtScanCounter < kSyncWords - kSyncTiles, "tile counter outside the kSyncTiles words");

template <int OP, typename T, int U>
__global__ __launch_bounds__(kScanThreads) void reduce_tiles_kernel(const T *__restrict__ x, size_t n, unsigned ntiles,
                                                                    unsigned per, scan_acc_t<OP, T> *local,
                                                                    scan_acc_t<OP, T> *block, scan_acc_t<OP, T> *bpart,
                                                                    unsigned *done, scan_acc_t<OP, T> *out) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  using OpC = Op<OP, C>;
  using OpA = Op<OP, A>;
  constexpr int V = Vec16<T>::N;
  constexpr int NW = kScanThreads / kWave;
  constexpr size_t TILE = (size_t)kScanThreads * U * V;
  constexpr int UL = U < 8 ? U : 8; // loads in flight per thread per step
  // per (tile, wave) folds of the current chunk of tiles, double-buffered:
  // wave 0 turns chunk k into prefixes while the other waves load chunk
  // k + 1 into the other buffer (one barrier per chunk)
  __shared__ A s_wb[2][kRtChunk][NW];
  __shared__ A s_red[NW];
  __shared__ bool s_last;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const unsigned t0 = blockIdx.x * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
  A run = OpA::identity(); // fold of this block's tiles so far (wave 0)
  unsigned ci = 0;
  for (unsigned c0 = t0; c0 < t1; c0 += kRtChunk, ci++) {
    const unsigned c1 = c0 + kRtChunk < t1 ? c0 + kRtChunk : t1;
    A(*s_w)[NW] = s_wb[ci & 1];
    unsigned t = c0;
    // small tiles (U < 8): TG whole tiles per step, all their loads issued
    // before any fold, so 8 loads per thread stay in flight as with U >= 8
    constexpr int TG = U >= 8 ? 1 : 8 / U;
    if constexpr (TG > 1) {
      if (((uintptr_t)x & 15) == 0) {
        for (; t + TG <= c1 && (size_t)(t + TG) * TILE <= n; t += TG) {
          const Vec16<T> *xv = reinterpret_cast<const Vec16<T> *>(x + (size_t)t * TILE);
          Vec16<T> v[TG][U];
#pragma unroll
          for (int g = 0; g < TG; g++)
#pragma unroll
            for (int u = 0; u < U; u++)
              v[g][u] = load_nt(xv + (size_t)g * (TILE / V) +
                                (wid * U + u) * kWave + lane);
          A acc[TG];
#pragma unroll
          for (int g = 0; g < TG; g++) {
            C f = OpC::identity();
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
              for (int j = 0; j < V; j++) f = OpC::apply(f, (C)v[g][u].v[j]);
            acc[g] = (A)f;
          }
#pragma unroll
          for (int g = 0; g < TG; g++) acc[g] = wave_reduce<OP>(acc[g]);
          if (lane == 0) {
#pragma unroll
            for (int g = 0; g < TG; g++) s_w[t + g - c0][wid] = acc[g];
          }
        }
      }
    }
    for (; t < c1; t++) {
      const size_t base = (size_t)t * TILE;
      A acc = OpA::identity();
      if (base + TILE <= n && ((uintptr_t)(x + base) & 15) == 0) {
        const Vec16<T> *xv = reinterpret_cast<const Vec16<T> *>(x + base);
#pragma unroll
        for (int u0 = 0; u0 < U; u0 += UL) {
          Vec16<T> v[UL];
#pragma unroll
          for (int u = 0; u < UL; u++)
            v[u] = load_nt(xv + (wid * U + u0 + u) * kWave + lane);
          C f = OpC::identity();
#pragma unroll
          for (int u = 0; u < UL; u++)
#pragma unroll
            for (int j = 0; j < V; j++) f = OpC::apply(f, (C)v[u].v[j]);
          acc = OpA::apply(acc, (A)f);
        }
      } else {
        // wave wid: its part [base + wid*Q, base + (wid+1)*Q) of the tile
        constexpr size_t Q = TILE / NW;
        const size_t b0 = base + (size_t)wid * Q, end = b0 + Q < n ? b0 + Q : n;
        for (size_t i = b0 + lane; i < end; i += kWave) acc = OpA::apply(acc, (A)(C)x[i]);
      }
      acc = wave_reduce<OP>(acc);
      if (lane == 0) s_w[t - c0][wid] = acc;
    }
    __syncthreads();
    if (wid == 0) {
      const unsigned k = lane;
      A agg = OpA::identity();
      if (c0 + k < c1) {
#pragma unroll
        for (int w = 0; w < NW; w++) agg = OpA::apply(agg, s_w[k][w]);
      }
      const A incl = wave_inclusive_scan<OP>(agg);
      const A ex = wave_shift_up1(incl, OpA::identity());
      // every wave part's exclusive prefix within the reduce block
      if (c0 + k < c1) {
        A p = OpA::apply(run, ex);
#pragma unroll
        for (int w = 0; w < NW; w++) {
          local[(size_t)(c0 + k) * NW + w] = p;
          p = OpA::apply(p, s_w[k][w]);
        }
      }
      run = OpA::apply(run, shfl_idx(incl, kWave - 1));
    }
  }
  // the block total (wave 0 holds it) -> two-level completion count; the
  // last block turns the block totals into block prefixes and the total
  if (tid == 0) {
    __hip_atomic_store(bpart + blockIdx.x, run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned g = blockIdx.x / 32, ng = (gridDim.x + 31) / 32;
    const unsigned in_g = gridDim.x - g * 32 < 32 ? gridDim.x - g * 32 : 32;
    bool last = __hip_atomic_fetch_add(done + (1 + g) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_g - 1;
    if (last) last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
    s_last = last;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  // thread i: block totals [i*q, (i+1)*q), left to right; then an exclusive
  // scan of the thread folds across the block
  const unsigned nb = gridDim.x, q = (nb + kScanThreads - 1) / kScanThreads;
  const unsigned b0 = tid * q < nb ? tid * q : nb, b1 = b0 + q < nb ? b0 + q : nb;
  A f = OpA::identity();
  for (unsigned b = b0; b < b1; b++)
    f = OpA::apply(f, __hip_atomic_load(bpart + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const A incl = wave_inclusive_scan<OP>(f);
  if (lane == kWave - 1) s_red[wid] = incl;
  __syncthreads();
  A pre = OpA::identity(), tot = OpA::identity();
#pragma unroll
  for (int w = 0; w < NW; w++) {
    if (w < wid) pre = OpA::apply(pre, s_red[w]);
    tot = OpA::apply(tot, s_red[w]);
  }
  A ex = OpA::apply(pre, wave_shift_up1(incl, OpA::identity()));
  for (unsigned b = b0; b < b1; b++) {
    block[b] = ex;
    ex = OpA::apply(ex, __hip_atomic_load(bpart + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  for (unsigned g = tid; g < (nb + 31) / 32; g += kScanThreads)
    __hip_atomic_store(done + (1 + g) * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid == 0) {
    *out = tot;
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// DRHIP_CHECK_TILES: a position-dependent 64-bit hash of the range's bits
// (XOR of mix(i, bits)), so a scan of a range changed since its reduce is
// caught; the compare kernel sets the segment's error word (4) on a mismatch
__device__ inline unsigned long long tiles_mix(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <typename T> __global__ void tiles_hash_kernel(const T *x, size_t n, unsigned long long *h) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long b = 0;
    __builtin_memcpy(&b, x + i, sizeof(T));
    acc ^= tiles_mix(b + 0x9E3779B97F4A7C15ull * (i + 1));
  }
  for (int m = 32; m >= 1; m >>= 1) acc ^= __shfl_xor(acc, m, 64);
  if ((threadIdx.x & 63) == 0) atomicXor(h, acc);
}
__global__ void tiles_hash_compare(const unsigned long long *h, unsigned *err) {
  if (h[0] != h[1]) __hip_atomic_store(err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T> static int launch_tiles_hash(Segment *s, const T *x, size_t n, unsigned long long *h) {
  DRHIP_CHECK_HIP(hipMemsetAsync(h, 0, sizeof(unsigned long long), s->stream));
  const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, (size_t)s->num_cus * 4));
  hipLaunchKernelGGL((tiles_hash_kernel<T>), dim3(grid), dim3(256), 0, s->stream, x, n, h);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

template <typename T, int OP, int UB>
static int launch_reduce_tiles(Segment *s, int seg, const T *x, size_t n, void *out) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  constexpr int U = scan_u<T, C, UB>();
  constexpr size_t TILE = (size_t)kScanThreads * U * V;
  const size_t ntiles = n ? (n + TILE - 1) / TILE : 0;
  if (ntiles > 0xFFFFFFF0ull) return set_error(DRHIP_ERR_BAD_ARG, "reduce_tiles: too many tiles");
  const unsigned cap = (unsigned)std::min<size_t>((size_t)s->num_cus * kRtBlocksPerCU, kRtMaxGrid);
  const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>(ntiles, cap));
  const unsigned per = ntiles ? (unsigned)((ntiles + grid - 1) / grid) : 1;
  const size_t nloc = ntiles * kTilesNW;
  const size_t need = (nloc + 2 * (size_t)grid) * sizeof(A) + 256;
  if (s->tiles_bytes < need) {
    if (int rc = may_reallocate(s, "drhip_reduce_tiles: the tile-prefix buffer")) return rc;
    s->tiles_bytes = 0;
    const size_t nb = (need + 4095) & ~size_t(4095);
    if (int rc = seg_realloc(s, &s->tiles, nb)) return rc;
    s->tiles_bytes = nb;
  }
  A *local = (A *)s->tiles, *block = local + nloc, *bpart = block + grid;
  s->tr = TilesRange{x, n, dtype_code_of<T>(), OP, per};
  if (s->capturing) {
    s->cap_tiles = true;
    s->tr_captured = s->tr;
  }
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (n == 0) {
    hipLaunchKernelGGL((write_scalar<A>), dim3(1), dim3(1), 0, s->stream, (A *)out, Op<OP, A>::identity());
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  }
  hipLaunchKernelGGL((reduce_tiles_kernel<OP, T, U>), dim3(grid), dim3(kScanThreads), 0, s->stream, x, n,
                     (unsigned)ntiles, per, local, block, bpart, s->dsync + kSyncTiles, (A *)out);
  DRHIP_CHECK_LAUNCH();
  if (s->check_tiles) return launch_tiles_hash<T>(s, x, n, s->thash);
  return DRHIP_OK;
}

template <typename T, int OP, int UB>
static int launch_scan_tiles(Segment *s, const T *in, T *out, size_t n, const void *carry_dev, const Gathered &g) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  constexpr int U = scan_u<T, C, UB>();
  constexpr size_t TILE = (size_t)kScanThreads * U * V;
  if (s->tr.x != (const void *)in || s->tr.n != n || s->tr.dtype != dtype_code_of<T>() || s->tr.op != OP)
    return set_error(DRHIP_ERR_BAD_ARG,
                     "drhip_inclusive_scan_tiles: not the range (pointer, size, dtype, op) of the segment's last "
                     "drhip_reduce_tiles");
  if (n == 0) {
    if (g.parts && g.result) {
      DRHIP_CHECK_HIP(hipSetDevice(s->device));
      return launch_fold_parts<OP, A>(s, g.parts, g.w, g.result);
    }
    return DRHIP_OK;
  }
  const size_t ntiles = (n + TILE - 1) / TILE;
  ScanArgs<A> a{};
  a.carry_dev = (const A *)carry_dev;
  a.parts = (const A *)g.parts;
  a.parts_w = g.w;
  a.parts_rank = g.rank;
  a.fold_res = (A *)g.result;
  a.err = s->err;
  a.tile_local = (const A *)s->tiles;
  a.tile_block = (const A *)s->tiles + ntiles * kTilesNW;
  a.tile_per = s->tr.per;
  a.tile_counter = s->dsync + kSyncTiles + kRtScanCounter;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (s->check_tiles) {
    if (int rc = launch_tiles_hash<T>(s, in, n, s->thash + 1)) return rc;
    hipLaunchKernelGGL(tiles_hash_compare, dim3(1), dim3(1), 0, s->stream, (const unsigned long long *)s->thash, s->err);
    DRHIP_CHECK_LAUNCH();
  }
  const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if (aligned)
    hipLaunchKernelGGL((scan_wave_given_kernel<OP, T, true, U>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, a);
  else
    hipLaunchKernelGGL((scan_wave_given_kernel<OP, T, false, U>), dim3((unsigned)ntiles), dim3(kScanThreads), 0,
                       s->stream, in, out, n, a);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

int scan_inclusive_u32(Segment *s, int seg, const uint32_t *in, uint32_t *out, size_t n) {
  return scan_dispatch<uint32_t, DRHIP_PLUS>(s, seg, in, out, n, nullptr, nullptr, nullptr, nullptr);
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
      return scan_dispatch<T, OP>(s, seg, (const T *)in, (T *)out, n, init_host, carry_host, carry_dev,
                                  total_acc);
    });
  });
}

extern "C" int drhip_inclusive_scan_gathered(int seg, int dtype, int op, const void *in, void *out, size_t n,
                                             const void *partials, int w, int rank, void *result) {
  DRHIP_GET_SEG(s, seg);
  if ((!in || !out) && n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan_gathered: null pointer");
  if (!partials || w < 1 || rank < 0 || rank >= w)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan_gathered: partials / w / rank");
  Gathered g;
  g.parts = partials;
  g.w = w;
  g.rank = rank;
  g.result = result;
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      return scan_dispatch<T, OP>(s, seg, (const T *)in, (T *)out, n, nullptr, nullptr, nullptr, nullptr, g);
    });
  });
}

extern "C" int drhip_reduce_tiles(int seg, int dtype, int op, const void *x, size_t n, void *out_acc) {
  DRHIP_GET_SEG(s, seg);
  if (!out_acc || (!x && n)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_reduce_tiles: null pointer");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      if (n * sizeof(T) >= kTilesBigBytes) return launch_reduce_tiles<T, OP, kTilesUBig>(s, seg, (const T *)x, n, out_acc);
      return launch_reduce_tiles<T, OP, kTilesU>(s, seg, (const T *)x, n, out_acc);
    });
  });
}

extern "C" int drhip_inclusive_scan_tiles(int seg, int dtype, int op, const void *in, void *out, size_t n,
                                          const void *carry_dev, const void *partials, int w, int rank,
                                          void *result) {
  DRHIP_GET_SEG(s, seg);
  if ((!in || !out) && n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan_tiles: null pointer");
  if (partials && (w < 1 || rank < 0 || rank >= w))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan_tiles: w / rank");
  Gathered g;
  g.parts = partials;
  g.w = w;
  g.rank = rank;
  g.result = result;
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      if (n * sizeof(T) >= kTilesBigBytes)
        return launch_scan_tiles<T, OP, kTilesUBig>(s, (const T *)in, (T *)out, n, carry_dev, g);
      return launch_scan_tiles<T, OP, kTilesU>(s, (const T *)in, (T *)out, n, carry_dev, g);
    });
  });
}
