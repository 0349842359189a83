// dr/shp/scan.hpp -- single-pass decoupled look-back scan for ANY operator
// and view (the template path of shp::inclusive_scan / exclusive_scan; the
// standard operators on arithmetic spans go to libdrhip's scan kernel).
//
// Reference semantics kept (include/dr/shp/algorithms/inclusive_scan.hpp):
//   * a zipped piece is scanned left to right with op(left, right); init
//     enters on the LEFT of piece 0's first element (:77-79, oneDPL
//     inclusive_scan with init);
//   * piece k > 0 receives the running fold S_{k-1} of the piece totals
//     (:108-116) on the RIGHT: x = op(x, S_{k-1}) (:132-134).  For a
//     non-commutative op this differs from std::inclusive_scan -- it is what
//     the reference computes, so it is what this computes.
// Only the ORDER of applications is a contract: op must be associative, as
// oneDPL requires.
//
// Kernel (one tile per workgroup, tile index from an atomic counter in start
// order, so every predecessor of a tile is already running):
//   tile = 256 threads x U slots x V elements; V consecutive elements per
//   slot when both ranges are 16-byte-aligned contiguous spans of T (one
//   16-B nontemporal load/store per slot), V = 1 through the accessors of
//   any other view (coalesced element loads);
//   in-thread scan of each slot's V elements; per-slot wave scan by DPP
//   row_shr / row_bcast moves, applied only where the source lane exists
//   (no identity element is needed); wave 0 scans the U x 4 piece totals in
//   element order and runs the look-back: the 64 lanes read 64 predecessor
//   status granules at once and fold them in tile order with an ordered
//   butterfly (higher lane = earlier tile on the left).
//   Status hand-off: T of <= 12 bytes is published as one self-validating
//   8-B word per 32 bits of T, {word, status}, each an 8-B agent-scope
//   atomic store / load (single-copy atomic; MI355X_MICROARCH "Valid forms"
//   R2: the value is the flag), accepted when every word carries the same
//   status (a tile's value is fixed per status); larger T uses separate aggregate /
//   inclusive value arrays written with sc1 stores, then s_waitcnt
//   vmcnt(0), then an sc1 status store, read back with sc1 loads after the
//   status poll matched (the guide's hand-off table, row 1).
// The last (partial) tile publishes nothing -- nothing waits on it -- so
// elements past n are loaded as copies of element n-1 and simply not
// stored.  8 B/elem moved for a 4-byte T (the round-1 template path was a
// 3-kernel reduce-then-scan at 12 B/elem).
#pragma once

#include <cstdint>
#include <type_traits>

#include "runtime.hpp"

namespace shp::detail {

constexpr int kLbThreads = 256;
constexpr int kLbWaves = kLbThreads / 64;
#ifndef DR_SHP_LB_SLOTS
#define DR_SHP_LB_SLOTS 32
#endif
constexpr int kLbSlots = DR_SHP_LB_SLOTS; // max U: slots per thread (wave 0 scans the U x 4 piece totals in chunks of 64)
// VGPRs budgeted for a thread's tile + lane prefixes (lb_slots)
#ifndef DR_SHP_LB_BUDGET
#define DR_SHP_LB_BUDGET 160
#endif
constexpr unsigned kLbSpinLimit = 1u << 22;
// DR_SHP_LB_BUF: full aligned tiles loaded with buffer loads, the slot
// offset in the SGPR soffset (one voffset VGPR for all U slots; a global
// load needs a 64-bit address per slot, u * 4 KiB exceeding the 13-bit
// immediate) -- the C-ABI scan's load (csrc/scan_kernel.hpp scan_load).
// Round 5, lambda-op scan of 2^29 f32 (tests/cpp/bin/dense_bench, three
// interleaved rounds on one box, profiles/r05_template_scan_ab.txt): global
// loads 0.692 / 0.694 / 0.701 of HBM, buffer loads 0.711 / 0.725 / 0.731,
// + early publication 0.714 / 0.726 / 0.733, + the fast combine 0.718 /
// 0.736 / 0.718 (the fast combine alone 0.703 / 0.718 / 0.716).
#ifndef DR_SHP_LB_BUF
#define DR_SHP_LB_BUF 1
#endif
// DR_SHP_LB_PUB: wave 0 publishes the tile aggregate as soon as the chunk
// scans have produced it, before the piece prefixes go to LDS.
#ifndef DR_SHP_LB_PUB
#define DR_SHP_LB_PUB 1
#endif
// DR_SHP_LB_FAST: the combine of a tile whose every piece has a prefix (a
// tile after the first, or one with a left carry) in a plain inclusive scan
// without a right carry: op(prefix, x) per element, no per-element
// "has a prefix" / carry selects (block-uniform branch).
#ifndef DR_SHP_LB_FAST
#define DR_SHP_LB_FAST 1
#endif
// DR_SHP_LB_EARLY: the tile aggregate as an ORDERED fold (per-slot wave
// folds in lane 63, then the pieces in element order), published before
// the per-slot wave scans -- the C-ABI scan's early aggregate without
// assuming a commutative operator (full tiles after the first).  Round 5,
// lambda-op scan of 2^29 f32, three interleaved rounds on one box
// (profiles/r05_template_scan_ab.txt): 0.720 / 0.709 / 0.719 without, 0.732
// / 0.743 / 0.745 with; the C++ suite's non-commutative scans (affine,
// affine3, mat2, keep-right) bit-exact with it.
#ifndef DR_SHP_LB_EARLY
#define DR_SHP_LB_EARLY 1
#endif
// DR_SHP_LB_EPOCH: no status reset per call.  Every status word carries the
// launch's epoch (tag = epoch << 2 | status, a word of another epoch reads
// as LB_NONE) and the tile counter is reset by the block that claims the
// last tile, so a call is one launch; the per-segment status buffer
// (runtime.hpp lb_status_pool) is cleared only on (re)allocation, layout
// switches and epoch wrap.  Round 5 (profiles/r05_template_scan_ab.txt, A/B
// #5 and #7): call-level 0.729-0.749 against 0.728-0.732 on one box, 0.740-
// 0.745 against 0.734-0.741 on another.  Its first stress runs exposed the
// stream-ordered pool's zero pages (profiles/r05_pool_stress.txt); on
// hipMalloc'd memory it ran 0 failures in 110 suite runs.
#ifndef DR_SHP_LB_EPOCH
#define DR_SHP_LB_EPOCH 1
#endif
// DR_SHP_LB_TEXC: wave 0 hands the look-back's prefix over in LDS and every
// thread folds it into its slots' piece prefixes in the combine, instead of
// wave 0 rewriting the NP piece prefixes before the barrier the other waves
// wait on.
#ifndef DR_SHP_LB_TEXC
#define DR_SHP_LB_TEXC 1
#endif
// DR_SHP_LB_PRIO: wave 0 runs the piece scan, look-back and publication at
// raised issue priority (s_setprio 3): the other waves of the tile wait on it.
#ifndef DR_SHP_LB_PRIO
#define DR_SHP_LB_PRIO 0
#endif

enum : unsigned { LB_NONE = 0, LB_AGG = 1, LB_INCL = 2 };

template <typename T> constexpr int lb_words = (sizeof(T) + 3) / 4;
template <typename T> constexpr bool lb_small = sizeof(T) <= 12; // value words tagged with the status
// one tile's granule per 128-B line: tiles publishing at the same time never
// share a line (the C-ABI scan's granule stride, csrc/scan_kernel.hpp
// kScanGStride: 8 -> 128 B per tile took 2^30 f32 1.51 -> 1.42 ms)
template <typename T> constexpr std::size_t lb_gran_bytes = (8 * ((sizeof(T) + 3) / 4) + 127) / 128 * 128;

template <typename T> struct lb_box {
  unsigned w[lb_words<T>];
};
template <typename T> __device__ __forceinline__ lb_box<T> lb_to_words(const T &x) {
  lb_box<T> b{};
  __builtin_memcpy(&b, &x, sizeof(T));
  return b;
}
template <typename T> __device__ __forceinline__ T lb_from_words(const lb_box<T> &b) {
  T x;
  __builtin_memcpy(&x, &b, sizeof(T));
  return x;
}

template <int CTRL, int ROW_MASK, typename T> __device__ __forceinline__ T lb_dpp(const T &old, const T &x) {
  const lb_box<T> o = lb_to_words(old), v = lb_to_words(x);
  lb_box<T> r;
#pragma unroll
  for (int i = 0; i < lb_words<T>; i++)
    r.w[i] = (unsigned)__builtin_amdgcn_update_dpp((int)o.w[i], (int)v.w[i], CTRL, ROW_MASK, 0xf, false);
  return lb_from_words<T>(r);
}
// DPP move with bound_ctrl and no `old` operand (lanes without a source get
// 0 or keep an undefined value) -- for lb_wave_fold_last, whose lane 63
// never depends on those lanes
template <int CTRL, int ROW_MASK, typename T> __device__ __forceinline__ T lb_dpp_nb(const T &x) {
  const lb_box<T> v = lb_to_words(x);
  lb_box<T> r;
#pragma unroll
  for (int i = 0; i < lb_words<T>; i++)
    r.w[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)v.w[i], CTRL, ROW_MASK, 0xf, true);
  return lb_from_words<T>(r);
}
template <typename T> __device__ __forceinline__ T lb_shfl_xor(const T &x, int m) {
  lb_box<T> v = lb_to_words(x);
#pragma unroll
  for (int i = 0; i < lb_words<T>; i++) v.w[i] = (unsigned)__shfl_xor((int)v.w[i], m, 64);
  return lb_from_words<T>(v);
}
template <typename T> __device__ __forceinline__ T lb_readlane(const T &x, int lane) {
  lb_box<T> v = lb_to_words(x);
#pragma unroll
  for (int i = 0; i < lb_words<T>; i++) v.w[i] = (unsigned)__builtin_amdgcn_readlane((int)v.w[i], lane);
  return lb_from_words<T>(v);
}

// Inclusive scan over the 64 lanes, op(earlier, later); a lane whose DPP
// source lies outside the row / wave keeps its value (no identity needed).
template <typename T, typename Op> __device__ __forceinline__ T lb_wave_scan(T x, const Op &op, int lane) {
  T y;
  y = lb_dpp<0x111, 0xf>(x, x); // row_shr:1
  if ((lane & 15) >= 1) x = static_cast<T>(op(y, x));
  y = lb_dpp<0x112, 0xf>(x, x); // row_shr:2
  if ((lane & 15) >= 2) x = static_cast<T>(op(y, x));
  y = lb_dpp<0x114, 0xf>(x, x); // row_shr:4
  if ((lane & 15) >= 4) x = static_cast<T>(op(y, x));
  y = lb_dpp<0x118, 0xf>(x, x); // row_shr:8
  if ((lane & 15) >= 8) x = static_cast<T>(op(y, x));
  y = lb_dpp<0x142, 0xa>(x, x); // row_bcast:15 -> rows 1, 3
  if (lane & 16) x = static_cast<T>(op(y, x));
  y = lb_dpp<0x143, 0xc>(x, x); // row_bcast:31 -> rows 2, 3
  if (lane & 32) x = static_cast<T>(op(y, x));
  return x;
}

// Ordered fold of the 64 lanes, op(earlier, later), in lane 63 (the other
// lanes end with partial or undefined values): the scan's six DPP steps
// without its selects -- every source lane 63 depends on exists at every
// step (row_shr 1/2/4/8 inside row 3, then row_bcast 15 / 31).
template <typename T, typename Op> __device__ __forceinline__ T lb_wave_fold_last(T x, const Op &op) {
  x = static_cast<T>(op(lb_dpp_nb<0x111, 0xf>(x), x));
  x = static_cast<T>(op(lb_dpp_nb<0x112, 0xf>(x), x));
  x = static_cast<T>(op(lb_dpp_nb<0x114, 0xf>(x), x));
  x = static_cast<T>(op(lb_dpp_nb<0x118, 0xf>(x), x));
  x = static_cast<T>(op(lb_dpp_nb<0x142, 0xa>(x), x));
  x = static_cast<T>(op(lb_dpp_nb<0x143, 0xc>(x), x));
  return x;
}

// Device-scope single-instruction stores / loads (see the file comment).
__device__ __forceinline__ void lb_store4_sc1(void *p, unsigned v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ unsigned lb_load4_sc1(const void *p) {
  unsigned r;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// Tile status of one launch.  small T: gran[t] = one 8-B {word, status}
// per value word; otherwise agg[t] / incl[t] value arrays plus stat[t].
template <typename T> struct lb_status {
  char *gran = nullptr;
  T *agg = nullptr;
  T *incl = nullptr;
  unsigned *stat = nullptr;
  unsigned epoch = 0; // tag = epoch << 2 | status (DR_SHP_LB_EPOCH; 0 after a reset)

  __device__ __forceinline__ unsigned decode(unsigned tag) const { return (tag >> 2) == epoch ? (tag & 3u) : LB_NONE; }

  __device__ void publish(std::size_t t, unsigned st, const T &v) const {
    const lb_box<T> b = lb_to_words(v);
    st |= epoch << 2;
    if constexpr (lb_small<T>) {
      auto *g = reinterpret_cast<std::uint64_t *>(gran + t * lb_gran_bytes<T>);
#pragma unroll
      for (int i = 0; i < lb_words<T>; i++)
        __hip_atomic_store(g + i, ((std::uint64_t)st << 32) | b.w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned *dst = reinterpret_cast<unsigned *>((st & 3u) == LB_AGG ? agg + t : incl + t);
#pragma unroll
      for (int i = 0; i < lb_words<T>; i++) lb_store4_sc1(dst + i, b.w[i]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lb_store4_sc1(stat + t, st);
    }
  }
  __device__ unsigned read(std::size_t t, T &v) const {
    lb_box<T> b;
    if constexpr (lb_small<T>) {
      const auto *g = reinterpret_cast<const std::uint64_t *>(gran + t * lb_gran_bytes<T>);
      std::uint64_t w[lb_words<T>];
#pragma unroll
      for (int i = 0; i < lb_words<T>; i++) w[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned tag = (unsigned)(w[0] >> 32);
      bool same = true;
#pragma unroll
      for (int i = 0; i < lb_words<T>; i++) {
        b.w[i] = (unsigned)w[i];
        same &= (unsigned)(w[i] >> 32) == tag;
      }
      v = lb_from_words<T>(b);
      return same ? decode(tag) : LB_NONE; // words of two different publications: not yet consistent
    } else {
      const unsigned st = decode(lb_load4_sc1(stat + t));
      if (st != LB_NONE) {
        const unsigned *src = reinterpret_cast<const unsigned *>(st == LB_AGG ? agg + t : incl + t);
#pragma unroll
        for (int i = 0; i < lb_words<T>; i++) b.w[i] = lb_load4_sc1(src + i);
        v = lb_from_words<T>(b);
      }
      return st;
    }
  }
};

template <typename T> struct lb_args {
  unsigned *counter;
  lb_status<T> status;
  bool has_l; // left carry: init of piece 0 (inclusive) / the piece's carry (exclusive)
  T lcarry;
  bool has_r; // right carry: S_{k-1} of inclusive_scan.hpp:132-134
  T rcarry;
  bool exclusive;
  bool reduce_only; // no output: only *total (the piece's fold, left carry included)
  T *total;         // nullable, device-visible
  unsigned *err;    // bounded-spin error word, device-visible
};

// Wave 0: ordered fold of every tile before `tile`; false when there is none.
template <typename T, typename Op>
__device__ bool lb_lookback(const lb_status<T> &g, long tile, int lane, const Op &op, T &excl, unsigned *err) {
  T acc{};
  bool has = false;
  long pred = tile - 1;
  unsigned spins = 0;
  while (true) {
    const long idx = pred - lane;
    T v{};
    unsigned st = LB_INCL; // before tile 0: an empty inclusive prefix
    bool valid = false;
    if (idx >= 0) {
      st = g.read(static_cast<std::size_t>(idx), v);
      valid = true;
    }
    const std::uint64_t incl = __ballot(st == LB_INCL);
    const int k = incl ? __builtin_ctzll(incl) : 64;
    const std::uint64_t upto = k >= 63 ? ~0ull : ((2ull << k) - 1ull);
    if (__ballot(st == LB_NONE) & upto) {
      if (++spins > kLbSpinLimit) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    bool ok = valid && lane <= k;
    // ordered butterfly: after the step of width m every lane holds the fold
    // of its aligned group of 2m lanes, the higher (earlier-tile) half left
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      const T pv = lb_shfl_xor(v, m);
      const bool pok = __shfl_xor(static_cast<int>(ok), m, 64) != 0;
      if (lane & m) {
        if (ok && pok) v = static_cast<T>(op(v, pv));
        else if (pok) v = pv;
      } else {
        if (ok && pok) v = static_cast<T>(op(pv, v));
        else if (pok) v = pv;
      }
      ok = ok || pok;
    }
    if (ok) {
      acc = has ? static_cast<T>(op(v, acc)) : v;
      has = true;
    }
    if (k < 64) break;
    pred -= 64;
  }
  excl = acc;
  return has;
}

// Slots per thread: the tile (U x V values) plus one lane prefix per slot
// kept near DR_SHP_LB_BUDGET VGPRs whatever the size of T (4-byte T: U = 32,
// 32 K-element tiles, 2 tiles per SIMD).  Round 3 (tools/gpu_r03k.sh, lambda
// scan of 2^29 f32): U = 32 0.768-0.789 ms against 0.828-0.835 ms for
// U = 16 at 4 tiles per SIMD -- more bytes per look-back wait, as in the
// C-ABI scan.
template <typename T, int V> constexpr int lb_slots() {
  constexpr int u = DR_SHP_LB_BUDGET / (lb_words<T> * (V + 1));
  return u < 2 ? 2 : u > kLbSlots ? kLbSlots : u;
}
template <typename T, int V, int U> constexpr int lb_min_waves() {
  return lb_words<T> <= 2 && U * lb_words<T> * (V + 1) <= 96 ? 4 : 2;
}

// One launch scans (or folds) one zipped piece.  VEC: In = const T*, Out =
// T* (both 16-B aligned contiguous spans), V = 16 / sizeof(T) elements per
// slot; otherwise In / Out are segment accessors and V = 1.
template <typename T, int V, int U, bool VEC, typename In, typename Out, typename Op>
__global__ __launch_bounds__(kLbThreads, (lb_min_waves<T, V, U>())) void lb_scan_kernel(In in, Out out, std::size_t n, Op op, lb_args<T> a) {
  constexpr int NT = kLbThreads, NW = kLbWaves, NP = U * NW;
  constexpr std::size_t TILE = (std::size_t)NT * U * V;
  __shared__ __attribute__((aligned(16))) unsigned char s_wt_raw[NP * sizeof(T)];
  __shared__ __attribute__((aligned(16))) unsigned char s_pre_raw[NP * sizeof(T)];
  __shared__ __attribute__((aligned(16))) unsigned char s_tot_raw[sizeof(T)];
  __shared__ bool s_has[NP];
  __shared__ bool s_fast;
  __shared__ bool s_th;                                    // DR_SHP_LB_TEXC: the tile has a prefix
  __shared__ __attribute__((aligned(16))) unsigned char s_tex_raw[sizeof(T)]; // ... and its value
  __shared__ __attribute__((aligned(16))) unsigned char s_er_raw[(DR_SHP_LB_EARLY ? NP : 1) * sizeof(T)];
  __shared__ unsigned s_tile;
  T *s_wt = reinterpret_cast<T *>(s_wt_raw);
  T *s_pre = reinterpret_cast<T *>(s_pre_raw);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    const unsigned t = atomicAdd(a.counter, 1u);
    // DR_SHP_LB_EPOCH: the last claim resets the counter for the next call
    // (every other block has claimed already; the next call on this stream
    // starts after this grid)
    if (DR_SHP_LB_EPOCH && t == gridDim.x - 1)
      __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const std::size_t tile = s_tile;
  const std::size_t ntiles = (n + TILE - 1) / TILE;
  if (tile >= ntiles) { // a counter that did not start at 0: report, touch nothing
    if (tid == 0) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const std::size_t base = tile * TILE;
  const bool full = base + TILE <= n;
  const std::size_t rem = full ? TILE : n - base;

  // ---- load: slot u of thread tid holds elements (u*NT + tid)*V + [0, V)
  T v[U][V];
  if constexpr (VEC) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const T *src = in + base;
    if (full && DR_SHP_LB_BUF) {
      const std::uint64_t ad = reinterpret_cast<std::uint64_t>(src);
      const std::uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(ad));
      const std::uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(ad >> 32));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void *>((static_cast<std::uint64_t>(hi) << 32) | lo), 0,
          static_cast<int>(TILE * sizeof(T)), 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const v4u w = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, u * NT * 16, 2 /* nt */);
        __builtin_memcpy(&v[u][0], &w, 16);
      }
    } else if (full) {
      const v4u *p = reinterpret_cast<const v4u *>(src);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const v4u w = __builtin_nontemporal_load(p + u * NT + tid);
        __builtin_memcpy(&v[u][0], &w, 16);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < V; j++) {
          const std::size_t li = ((std::size_t)u * NT + tid) * V + j;
          v[u][j] = src[li < rem ? li : rem - 1];
        }
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const std::size_t li = (std::size_t)u * NT + tid;
      v[u][0] = static_cast<T>(in(base + (li < rem ? li : rem - 1)));
    }
  }

  // ---- in-thread scan of each slot, wave scans of the slot totals
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 1; j < V; j++) v[u][j] = static_cast<T>(op(v[u][j - 1], v[u][j]));
  // ---- early aggregate (DR_SHP_LB_EARLY): ordered, published by wave 0
  //      before the wave scans below
  constexpr bool EARLY = DR_SHP_LB_EARLY;
  const bool early = EARLY && full && tile != 0; // block-uniform
  T eagg{};
  if constexpr (EARLY) {
    if (early) {
      T *s_er = reinterpret_cast<T *>(s_er_raw);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const T r = lb_wave_fold_last(v[u][V - 1], op);
        if (lane == 63) s_er[u * NW + wid] = r;
      }
      __syncthreads();
      if (wid == 0) {
#pragma unroll
        for (int c0 = 0; c0 < NP; c0 += 64) {
          // a partial last chunk (NP not a multiple of 64): the masked scan,
          // read at its last valid lane
          const int cnt = NP - c0 < 64 ? NP - c0 : 64;
          const T pt = s_er[c0 + lane < NP ? c0 + lane : NP - 1];
          const T ct = cnt == 64 ? lb_readlane(lb_wave_fold_last(pt, op), 63)
                                 : lb_readlane(lb_wave_scan(pt, op, lane), cnt - 1);
          eagg = c0 == 0 ? ct : static_cast<T>(op(eagg, ct));
        }
        if (lane == 0) a.status.publish(tile, LB_AGG, eagg);
      }
    }
  }
  T lx[U]; // becomes the lane's exclusive prefix inside its wave (lane 0: none)
#pragma unroll
  for (int u = 0; u < U; u++) {
    lx[u] = lb_wave_scan(v[u][V - 1], op, lane);
    if (lane == 63) s_wt[u * NW + wid] = lx[u];
    lx[u] = lb_dpp<0x138, 0xf>(lx[u], lx[u]); // wave_shr:1
  }
  __syncthreads();

  // ---- wave 0: piece prefixes (in chunks of 64 pieces), tile aggregate,
  //      look-back, publication
  if (wid == 0) {
    if constexpr (DR_SHP_LB_PRIO) __builtin_amdgcn_s_setprio(3);
    T agg{};
    bool ah = false; // agg holds the fold of the chunks so far
    constexpr int NC = (NP + 63) / 64;
    T pins[NC], aggs[NC]; // DR_SHP_LB_PUB: each chunk's scan and the fold before it
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const int c0 = c * 64, idx = c0 + lane;
      const T pt = s_wt[idx < NP ? idx : NP - 1];
      const T pin = lb_wave_scan(pt, op, lane);
      if constexpr (DR_SHP_LB_PUB) {
        pins[c] = pin;
        aggs[c] = agg;
      } else {
        const T pex = lb_dpp<0x138, 0xf>(pin, pin); // lane l > 0: this chunk's pieces before l
        T p = pex;
        bool ph = lane > 0;
        if (ah) {
          p = ph ? static_cast<T>(op(agg, pex)) : agg;
          ph = true;
        }
        if (idx < NP) {
          s_pre[idx] = p;
          s_has[idx] = ph;
        }
      }
      const T ctot = lb_readlane(pin, (NP - c0 < 64 ? NP - c0 : 64) - 1);
      agg = ah ? static_cast<T>(op(agg, ctot)) : ctot;
      ah = true;
    }
    if (early) agg = eagg; // the value already published
    if constexpr (DR_SHP_LB_PUB)
      if (!early && tile != 0 && full && lane == 0) a.status.publish(tile, LB_AGG, agg);
    if constexpr (DR_SHP_LB_PUB) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const int idx = c * 64 + lane;
        const T pex = lb_dpp<0x138, 0xf>(pins[c], pins[c]);
        T p = pex;
        bool ph = lane > 0;
        if (c > 0) {
          p = ph ? static_cast<T>(op(aggs[c], pex)) : aggs[c];
          ph = true;
        }
        if (idx < NP) {
          s_pre[idx] = p;
          s_has[idx] = ph;
        }
      }
    }
    T tex{};
    bool th = false;
    if (tile == 0) {
      if (a.has_l) {
        tex = a.lcarry;
        th = true;
      }
      if (full && lane == 0) a.status.publish(0, LB_INCL, th ? static_cast<T>(op(tex, agg)) : agg);
    } else {
      if (!DR_SHP_LB_PUB && !early && full && lane == 0) a.status.publish(tile, LB_AGG, agg);
      th = lb_lookback(a.status, static_cast<long>(tile), lane, op, tex, a.err);
      if (full && lane == 0) a.status.publish(tile, LB_INCL, th ? static_cast<T>(op(tex, agg)) : agg);
    }
    if (DR_SHP_LB_TEXC) {
      if (lane == 0) {
        s_th = th;
        *reinterpret_cast<T *>(s_tex_raw) = tex;
      }
    } else if (th) {
#pragma unroll
      for (int c0 = 0; c0 < NP; c0 += 64) {
        const int idx = c0 + lane;
        if (idx < NP) {
          s_pre[idx] = s_has[idx] ? static_cast<T>(op(tex, s_pre[idx])) : tex;
          s_has[idx] = true;
        }
      }
    }
    if (full && tile == ntiles - 1 && lane == 0 && a.total) *a.total = th ? static_cast<T>(op(tex, agg)) : agg;
    if (lane == 0) s_fast = DR_SHP_LB_FAST && th && full && !a.exclusive && !a.has_r && !a.reduce_only;
    if constexpr (DR_SHP_LB_PRIO) __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  if constexpr (DR_SHP_LB_FAST) {
    if (s_fast) {
      // every piece has a prefix: s_pre[p] = fold of everything before piece
      // p; lane l > 0 adds its wave-exclusive prefix lx
      const T tx = *reinterpret_cast<const T *>(s_tex_raw);
#pragma unroll
      for (int u = 0; u < U; u++) {
        T sp = s_pre[u * NW + wid];
        if constexpr (DR_SHP_LB_TEXC) sp = s_has[u * NW + wid] ? static_cast<T>(op(tx, sp)) : tx;
        const T pp = lane > 0 ? static_cast<T>(op(sp, lx[u])) : sp;
        T r[V];
#pragma unroll
        for (int j = 0; j < V; j++) r[j] = static_cast<T>(op(pp, v[u][j]));
        if constexpr (VEC) {
          typedef unsigned v4u __attribute__((ext_vector_type(4)));
          v4u w;
          __builtin_memcpy(&w, r, 16);
          __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(out + base) + u * NT + tid);
        } else {
          out(base + (std::size_t)u * NT + tid) = r[0];
        }
      }
      return;
    }
  }

  // ---- combine (and store)
  const std::size_t last = rem - 1; // element whose inclusive value is the partial tile's total
#pragma unroll
  for (int u = 0; u < U; u++) {
    T sp = s_pre[u * NW + wid];
    bool sh = s_has[u * NW + wid];
    if (DR_SHP_LB_TEXC && s_th) {
      sp = sh ? static_cast<T>(op(*reinterpret_cast<const T *>(s_tex_raw), sp)) : *reinterpret_cast<const T *>(s_tex_raw);
      sh = true;
    }
    T pp = lx[u];
    bool ph = lane > 0;
    if (sh) {
      pp = ph ? static_cast<T>(op(sp, lx[u])) : sp;
      ph = true;
    }
    T r[V];
#pragma unroll
    for (int j = 0; j < V; j++) {
      const T inc = ph ? static_cast<T>(op(pp, v[u][j])) : v[u][j];
      if (!full) {
        const std::size_t li = ((std::size_t)u * NT + tid) * V + j;
        if (li == last) *reinterpret_cast<T *>(s_tot_raw) = inc;
      }
      if (a.exclusive) {
        // std::exclusive_scan: the fold of everything before the element
        // (a left carry always exists: init)
        r[j] = j == 0 ? pp : (ph ? static_cast<T>(op(pp, v[u][j - 1])) : v[u][j - 1]);
      } else {
        r[j] = a.has_r ? static_cast<T>(op(inc, a.rcarry)) : inc;
      }
    }
    if (a.reduce_only) continue;
    if constexpr (VEC) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      T *dst = out + base;
      if (full) {
        v4u w;
        __builtin_memcpy(&w, r, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(dst) + u * NT + tid);
      } else {
#pragma unroll
        for (int j = 0; j < V; j++) {
          const std::size_t li = ((std::size_t)u * NT + tid) * V + j;
          if (li < rem) dst[li] = r[j];
        }
      }
    } else {
      const std::size_t li = (std::size_t)u * NT + tid;
      if (li < rem) out(base + li) = r[0];
    }
  }
  if (!full) {
    __syncthreads();
    if (tid == 0 && a.total) *a.total = *reinterpret_cast<const T *>(s_tot_raw);
  }
}

// ------------------------------------------------------------------ host

template <typename T> constexpr bool lb_vec_type = std::is_trivially_copyable_v<T> &&
                                                   (sizeof(T) == 4 || sizeof(T) == 8 || sizeof(T) == 16);

// Enqueue one look-back scan of `in` (-> `out` unless reduce_only) on the
// stream of in's segment.  `total` / `err` must be device-visible (pinned).
template <typename T, typename SI, typename SO, typename Op>
void lb_scan_launch(const SI &in, const SO &out, Op op, bool has_l, T lcarry, bool has_r, T rcarry, bool exclusive,
                    bool reduce_only, T *total, unsigned *err) {
  const std::size_t n = in.size();
  if (n == 0) return;
  const std::size_t rank = in.rank();
  hipStream_t st = stream(rank);

  auto run = [&](auto v_tag, auto vec_tag, auto in_acc, auto out_acc) {
    constexpr int V = decltype(v_tag)::value;
    constexpr bool VEC = decltype(vec_tag)::value;
    constexpr int U = lb_slots<T, V>();
    const std::size_t tile = (std::size_t)kLbThreads * U * V;
    const std::size_t ntiles = (n + tile - 1) / tile;
    const std::size_t head = 256; // tile counter
    const std::size_t stat_bytes = lb_small<T> ? ntiles * lb_gran_bytes<T> : ntiles * sizeof(unsigned);
    const std::size_t val_bytes = lb_small<T> ? 0 : 2 * ntiles * ((sizeof(T) + 15) & ~std::size_t(15));
    // the value arrays start at the next 256-B boundary after the status words
    const std::size_t span = head + ((stat_bytes + 255) & ~std::size_t(255)) + val_bytes;
    char *ws = nullptr;
    unsigned epoch = 0;
    if constexpr (DR_SHP_LB_EPOCH) {
      ws = static_cast<char *>(lb_status_buffers().get(rank, span, head + stat_bytes,
                                                      !lb_small<T>, st, epoch));
    } else {
      ws = static_cast<char *>(device_scratch().get(rank, span));
    }
    lb_args<T> a{};
    a.status.epoch = epoch;
    a.counter = reinterpret_cast<unsigned *>(ws);
    if constexpr (lb_small<T>) {
      a.status.gran = ws + head;
    } else {
      a.status.stat = reinterpret_cast<unsigned *>(ws + head);
      char *vals = ws + head + ((stat_bytes + 255) & ~std::size_t(255));
      a.status.agg = reinterpret_cast<T *>(vals);
      a.status.incl = a.status.agg + ntiles;
    }
    a.has_l = has_l;
    a.lcarry = lcarry;
    a.has_r = has_r;
    a.rcarry = rcarry;
    a.exclusive = exclusive;
    a.reduce_only = reduce_only;
    a.total = total;
    a.err = err;
    if constexpr (!DR_SHP_LB_EPOCH) hip_check(hipMemsetAsync(ws, 0, head + stat_bytes, st), "scan status reset");
    hipLaunchKernelGGL((lb_scan_kernel<T, V, U, VEC, decltype(in_acc), decltype(out_acc), Op>),
                       dim3(static_cast<unsigned>(ntiles)), dim3(kLbThreads), 0, st, in_acc, out_acc, n, op, a);
    hip_check(hipGetLastError(), "look-back scan launch");
  };

  if constexpr (is_device_span<SI> && is_device_span<SO>) {
    using EI = std::remove_const_t<typename SI::value_type>;
    using EO = std::remove_const_t<typename SO::value_type>;
    if constexpr (std::is_same_v<EI, T> && std::is_same_v<EO, T> && lb_vec_type<T>) {
      const bool aligned = reinterpret_cast<std::uintptr_t>(in.data()) % 16 == 0 &&
                           (reduce_only || reinterpret_cast<std::uintptr_t>(out.data()) % 16 == 0);
      if (aligned) {
        run(std::integral_constant<int, 16 / sizeof(T)>{}, std::true_type{}, static_cast<const T *>(in.data()),
            reduce_only ? static_cast<T *>(nullptr) : const_cast<T *>(out.data()));
        return;
      }
    }
  }
  run(std::integral_constant<int, 1>{}, std::false_type{}, accessor_of(in), accessor_of(out));
}

} // namespace shp::detail
