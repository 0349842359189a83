// scan_kernel.hpp -- single-pass inclusive scan (decoupled look-back) for gfx950.
// Device code only; the launcher and C-ABI entry are in scan.hip.
//
// Replaces phases 1 and 3 of shp::inclusive_scan
// (include/dr/shp/algorithms/inclusive_scan.hpp:77-83 oneDPL
// inclusive_scan_async per zipped piece + :85-96 single_task copy of the
// piece's last value; :118-143 a SECOND full pass x = op(x, carry) with
// oneDPL for_each_async).  Here the carry is folded in-flight: one read and
// one write per element (8 B/elem for 4-byte types) instead of ~16.
//
// Tile = 256 threads x U vectors x 16 B (U = 8: 8192 f32/i32 = 32 KiB).
//   1. tile index from an atomic counter (dispatch order is not a contract
//      on gfx950, so tiles are numbered in the order blocks START; every
//      predecessor of a tile is then already running -> forward progress);
//   2. U independent 16-byte loads per thread (1 KiB per wave-instruction);
//   3. per-vector serial scan, U interleaved DPP wave scans, wave
//      totals through LDS -> tile aggregate;
//   4. wave 0 publishes the aggregate and looks back over 64 predecessor
//      tiles per step (one granule per lane, ballot, wave reduce), then
//      publishes its inclusive prefix;
//   5. every element: out = excl (ACC) op local (fp32 in-tile for f32 plus,
//      fp64 inter-tile carries: SURVEY.md 8d tolerance analysis).
// Inter-workgroup hand-off: MI355X_MICROARCH "Valid forms" R2 -- the value
// IS the flag.  Each tile owns one granule of self-validating 8-byte words,
// every word written by ONE 8-B agent-scope atomic store and read by ONE 8-B
// atomic load (single-copy atomic for an aligned 8-B atomic: an
// architectural guarantee), each word carrying a status / valid tag next
// to 32 bits of the value: 4-byte ACC {value, status}; 8-byte ACC the lo
// and hi words of the aggregate and of the inclusive value, each written
// once, a value accepted only when both its words are valid (see
// Granules).  No payload/flag ordering exists to get wrong, and no 16-byte
// access is assumed untorn.  Granules are zeroed by a memset node before
// every launch; every spin is bounded and reports through the segment's
// error word.
#pragma once
#include "common.hpp"

#include <type_traits>

namespace drhip {

constexpr int kScanThreads = 256;
constexpr int kScanWaves = kScanThreads / kWave;
constexpr int kScanU = 16;    // vectors per thread below kScanBigBytes (64 KiB tiles, 4 blocks/CU)
#ifndef DRHIP_SCAN_UBIG
#define DRHIP_SCAN_UBIG 32
#endif
constexpr int kScanUBig = DRHIP_SCAN_UBIG; // from kScanBigBytes up: 128 KiB tiles, 2 blocks/CU
constexpr size_t kScanBigBytes = size_t(1) << 27;
// Vectors per thread for element type T computed in C: UB x 16 B of data
// registers, halved when the compute type is wider than the element
// (fp32 products in fp64) so the tile stays within the VGPR budget.
// tools/scan_sweep.hip, 2^30 f32: U = 16 1.66 ms (look-back waits ~6.6 us
// per tile, 40 % of a tile's life), U = 32 1.50 ms (same wait, twice the
// bytes per wait), U = 48 / 64 spill to AGPRs and lose (1.61 ms).
template <typename T, typename C, int UB = kScanU> constexpr int scan_u() {
  return sizeof(C) > sizeof(T) ? UB / 2 : UB;
}

// Variant bits (tools/scan_sweep.hip measures them; product uses kScanFlags).
enum : int { SCAN_F32_COMBINE = 1, SCAN_NT_STORE = 2, SCAN_NO_LOOKBACK = 4, SCAN_LB4 = 8, SCAN_DIAG = 16,
             SCAN_NT_LOAD = 32, SCAN_PERSIST = 64, SCAN_BUF_LOAD = 128, SCAN_BUF_STORE = 256,
             SCAN_BUFFER = SCAN_BUF_LOAD | SCAN_BUF_STORE, SCAN_EARLY_AGG = 512, SCAN_EARLY_LB = 1024 };
// Output written once and input read once: nontemporal both ways; buffer
// loads keep the U slot offsets in SGPRs.  Buffer STORES (SCAN_BUF_STORE)
// are not used: with them, at U = 32, the 4th dword of lanes 12-15 of some
// rows intermittently landed wrong in memory (tools/dbg_scan.py: ~400 bad
// elements per 2^27; global stores, or buffer loads alone, 0 bad).
// SCAN_EARLY_AGG (every C-ABI operator is commutative): tools/scan_sweep.hip
// mode 4, 2^30 f32: 1.472 -> 1.421 ms; look-back 6.3 -> 4.4 us per tile,
// polls that found a predecessor unpublished 3.2 -> 1.7.
#ifndef DRHIP_SCAN_FLAGS
#define DRHIP_SCAN_FLAGS (SCAN_NT_STORE | SCAN_NT_LOAD | SCAN_BUF_LOAD | SCAN_EARLY_AGG)
#endif
constexpr int kScanFlags = DRHIP_SCAN_FLAGS;
constexpr int kScanMinW = 1; // __launch_bounds__ waves per SIMD
constexpr unsigned kSpinLimit = 1u << 22;

// In-tile compute type: fp32 stays fp32 for +,min,max (tile error is
// O(log tile) roundings); fp32 products are fp64 (compute_of, common.hpp).
template <int OP, typename T> using scan_c_t = typename compute_of<OP, T>::type;
template <int OP, typename T>
using scan_acc_t = std::conditional_t<std::is_floating_point_v<T>, double,
                                      typename compute_of<OP, T>::type>;

enum : unsigned { ST_NONE = 0, ST_AGG = 1, ST_INCL = 2 };


// One granule per tile.  4-byte ACC: u64 {status:32 | value:32}, AGG
// then INCL overwriting it in one 8-B store.  8-byte ACC: four word arrays
// (quarters of the granule array), each word {valid:32 | 32 value bits}
// written ONCE per launch: aggregate lo / hi and inclusive lo / hi.  A
// reader takes the inclusive value when both its words are valid, else the
// aggregate when both of those are, else nothing yet -- so a successor that
// polls while a tile's two INCL stores are landing falls back to the AGG
// published long before instead of re-polling (with ONE overwritten pair of
// words the half-landed INCL cost a full re-poll on the critical path:
// 1.596 vs 1.467 ms at 2^30 f32, gpurun r03b).
//
// P62 (fp64 ACC of fp32 data -- the C2 scan): ONE 8-B word per tile, the
// double with its two lowest mantissa bits replaced by the status
// ({value:62 | status:2}), one atomic store per publication, AGG overwritten
// by INCL.  Dropping 2 of 52 mantissa bits perturbs an inter-tile prefix by
// <= 2^-50 relative (a tile's fp32 aggregate is exact: 29 trailing zero
// bits), far below the fp32 outputs' resolution (2^-24); 8 B per tile, so a
// look-back step of 64 tiles reads 4 lines.
// One-word forms (P62, 4-byte ACC): one word per kScanGStride bytes.
// DRHIP_SCAN_GSTRIDE (bytes, a multiple of 8): the default is set by the
// measurement in DESIGN.md section 4 (scan notes).
#ifndef DRHIP_SCAN_GSTRIDE
#define DRHIP_SCAN_GSTRIDE 128
#endif
constexpr size_t kScanGStride = DRHIP_SCAN_GSTRIDE;
static_assert(kScanGStride % 8 == 0, "granule stride: whole 8-byte words");
template <typename A, bool P62 = false> struct Granules {
  char *base;
  int bytes; // granule array size (bytes)
  __device__ __forceinline__ uint64_t *word(long t) const { return (uint64_t *)(base + (size_t)t * kScanGStride); }

  __device__ __forceinline__ uint64_t *words(int k) const { return (uint64_t *)(base + (size_t)k * (bytes >> 2)); }
  __device__ __forceinline__ void publish(long t, unsigned status, A v) const {
    if constexpr (P62) {
      static_assert(sizeof(A) == 8, "P62: 8-byte ACC");
      uint64_t bits;
      __builtin_memcpy(&bits, &v, 8);
      __hip_atomic_store(word(t), (bits & ~3ull) | status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (sizeof(A) == 4) {
      uint32_t bits;
      __builtin_memcpy(&bits, &v, 4);
      __hip_atomic_store(word(t), ((uint64_t)status << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      uint64_t bits;
      __builtin_memcpy(&bits, &v, 8);
      const int k = status == ST_INCL ? 2 : 0;
      __hip_atomic_store(words(k) + t, (1ull << 32) | (uint32_t)bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(words(k + 1) + t, (1ull << 32) | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // status of tile t and its value (ST_NONE: nothing complete yet)
  __device__ __forceinline__ unsigned read(long t, A &v) const {
    if constexpr (P62) {
      const uint64_t w = __hip_atomic_load(word(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t bits = w & ~3ull;
      __builtin_memcpy(&v, &bits, 8);
      return (unsigned)(w & 3u);
    } else if constexpr (sizeof(A) == 4) {
      const uint64_t w = __hip_atomic_load(word(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t bits = (uint32_t)w;
      __builtin_memcpy(&v, &bits, 4);
      return (unsigned)(w >> 32);
    } else {
      const uint64_t al = __hip_atomic_load(words(0) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t ah = __hip_atomic_load(words(1) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t il = __hip_atomic_load(words(2) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t ih = __hip_atomic_load(words(3) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool incl = (il >> 32) && (ih >> 32), agg = (al >> 32) && (ah >> 32);
      const uint64_t bits = incl ? ((ih << 32) | (uint32_t)il) : ((ah << 32) | (uint32_t)al);
      __builtin_memcpy(&v, &bits, 8);
      return incl ? (unsigned)ST_INCL : agg ? (unsigned)ST_AGG : (unsigned)ST_NONE;
    }
  }
};

template <int OP, typename T>
using granules_t = Granules<scan_acc_t<OP, T>, std::is_same_v<T, float> && sizeof(scan_acc_t<OP, T>) == 8>;
// bytes per tile of granules_t
template <int OP, typename T> constexpr size_t granule_bytes() {
  return (std::is_same_v<T, float> || sizeof(scan_acc_t<OP, T>) == 4) ? kScanGStride : 32;
}

// Buffer resource over one tile; the base is block-uniform (readfirstlane
// keeps it in SGPRs, no waterfall loop).
template <typename T> __device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const T *p, size_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, (int)bytes, 0x00020000);
}

template <typename A> struct ScanArgs {
  int has_carry;
  A carry;
  const A *carry_dev;
  // drhip_inclusive_scan_gathered: the w gathered segment totals; tile 0
  // folds those of ranks < parts_rank into its carry and all w into
  // *fold_res, in drhip_fold_partials' order (one kernel fewer per step)
  const A *parts;
  int parts_w, parts_rank;
  A *fold_res;
  // scan_wave_given_kernel: the part prefixes of drhip_reduce_tiles
  const A *tile_local;
  const A *tile_block;
  unsigned tile_per;
  unsigned *tile_counter; // big tiles claimed in start order (self-resetting)
  A *total;
  unsigned *err;
  unsigned long long *diag; // SCAN_DIAG builds only: 8 words per tile
};

// Wave-0 look-back: returns op-fold of every tile before `tile`.
// One step examines W*64 predecessors (W independent granule loads per
// lane, distance d = w*64 + lane), so the INCL frontier -- about as many
// tiles back as are resident on the chip -- is reached in few dependent
// round trips.
template <int OP, typename A, int W, typename G>
__device__ A lookback(const G &g, long tile, int lane, unsigned *err, unsigned *nsteps = nullptr,
                     unsigned *nspins = nullptr) {
  using OpA = Op<OP, A>;
  A excl = OpA::identity();
  long pred = tile - 1;
  unsigned spins = 0, steps = 0;
  while (true) {
    A v[W];
    unsigned st[W];
#pragma unroll
    for (int w = 0; w < W; w++) {
      const long idx = pred - (w * kWave + lane);
      v[w] = OpA::identity();
      st[w] = ST_INCL; // tiles before 0: an inclusive identity
      if (idx >= 0) st[w] = g.read(idx, v[w]);
    }
    // first INCL by distance, and whether any nearer granule is unset
    int k = W * kWave;
    bool none_before = false;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint64_t incl_mask = __ballot(st[w] == ST_INCL);
      const uint64_t none_mask = __ballot(st[w] == ST_NONE);
      if (k == W * kWave) {
        const int kw = incl_mask ? __builtin_ctzll(incl_mask) : kWave;
        const uint64_t upto = kw == kWave ? ~0ull : ((2ull << kw) - 1ull); // lanes 0..kw
        none_before |= (none_mask & upto) != 0;
        if (kw < kWave) k = w * kWave + kw;
      }
    }
    if (none_before) {
      if (++spins > kSpinLimit) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory"); // re-read every granule next pass
      continue;
    }
    A f = OpA::identity();
#pragma unroll
    for (int w = 0; w < W; w++)
      if (w * kWave + lane <= k) f = OpA::apply(f, v[w]);
    f = wave_reduce<OP>(f);
    excl = OpA::apply(f, excl);
    steps++;
    if (k < W * kWave) break;
    pred -= W * kWave;
  }
  if (nsteps) *nsteps = steps;
  if (nspins) *nspins = spins;
  return excl;
}

// Register-lean body: the tile lives in ONE register array (U x 16 B per
// lane) that is scanned in place; per vector slot only one extra register
// (the wave-scan value, then the thread's exclusive prefix) is live, so
// U = 16 fits the 128-VGPR budget of 4 resident blocks per CU.
template <int OP, typename T, int U, int NT = kScanThreads> struct ScanSmem {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  C s_wt[U][NT / kWave];
  C s_pre[U][NT / kWave];
  C s_early[NT / kWave]; // SCAN_EARLY_AGG: per-wave folds of the tile
  A s_excl;
  unsigned s_tile;
  unsigned s_next;
};

// The tile's loads (16 B per lane per slot; OOB elements of the last tile =
// identity) into the register array v.
template <int OP, typename T, bool ALIGNED, int U, int FLAGS, int NT = kScanThreads>
__device__ __forceinline__ void scan_load(const T *in, size_t n, size_t tile,
                                          scan_c_t<OP, T> (&v)[U][Vec16<T>::N]) {
  using C = scan_c_t<OP, T>;
  using OpC = Op<OP, C>;
  constexpr int V = Vec16<T>::N;
  constexpr size_t TILE = (size_t)NT * U * V;
  const int tid = threadIdx.x;
  const size_t base = tile * TILE;
  const bool full = base + TILE <= n;
  if (ALIGNED && full && (FLAGS & SCAN_BUF_LOAD)) {
    // buffer loads: one voffset VGPR (tid*16) for all U slots, the slot
    // offset in the SGPR soffset -- global loads need a 64-bit address per
    // slot (u*4 KiB exceeds the 13-bit immediate), 2U VGPRs
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(in + base, TILE * sizeof(T));
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 raw = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, u * NT * 16,
                                                              (FLAGS & SCAN_NT_LOAD) ? 2 /* nt */ : 0);
      Vec16<T> r;
      __builtin_memcpy(&r, &raw, 16);
#pragma unroll
      for (int j = 0; j < V; j++) v[u][j] = (C)r.v[j];
    }
  } else if (ALIGNED && full) {
    const Vec16<T> *src = reinterpret_cast<const Vec16<T> *>(in + base);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const Vec16<T> r = (FLAGS & SCAN_NT_LOAD) ? load_nt(src + u * NT + tid) : src[u * NT + tid];
#pragma unroll
      for (int j = 0; j < V; j++) v[u][j] = (C)r.v[j];
    }
  } else {
    // partial or unaligned tile: uniform base pointer + 32-bit offsets
    const T *src = in + base;
    const unsigned rem = (unsigned)(n - base < TILE ? n - base : TILE);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * NT + tid) * V + j;
        v[u][j] = li < rem ? (C)src[li] : OpC::identity();
        // keep the (rare) partial-tile loads from being hoisted together:
        // their 64 address/result registers would set the whole kernel's
        // VGPR budget
        __builtin_amdgcn_sched_barrier(0);
      }
  }
}

// The rest of a tile once its registers hold the data: in-tile scans, the
// exclusive prefix (carry / look-back), the combine and the stores.
// hand_next: wave 0 hands `nxt` over in sm.s_next between the two barriers.
template <int OP, typename T, bool ALIGNED, int U, int FLAGS, int NT = kScanThreads>
__device__ __forceinline__ void scan_body(T *out, size_t n, size_t tile, scan_c_t<OP, T> (&v)[U][Vec16<T>::N],
                                          bool hand_next, unsigned nxt,
                                          const granules_t<OP, T> &gr, const ScanArgs<scan_acc_t<OP, T>> &a,
                                          ScanSmem<OP, T, U, NT> &sm) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  using OpC = Op<OP, C>;
  using OpA = Op<OP, A>;
  constexpr int V = Vec16<T>::N;
  constexpr size_t TILE = (size_t)NT * U * V;
  constexpr int LBW = (FLAGS & SCAN_LB4) ? 4 : 1;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wid = tid / kWave;
  const size_t ntiles = (n + TILE - 1) / TILE;
  const size_t base = tile * TILE;
  const bool full = base + TILE <= n;
  // wave 0: the tile's exclusive prefix (carry or look-back), its INCL
  // publication and the hand-over through LDS
  auto resolve = [&](C agg) {
    A excl;
    if (tile == 0) {
      excl = OpA::identity();
      if (a.has_carry) excl = a.carry;
      if (a.carry_dev) excl = OpA::apply(excl, *a.carry_dev);
      if (a.parts) {
        A acc = a.parts[0], c = acc;
        for (int k = 1; k < a.parts_w; k++) {
          if (k == a.parts_rank) c = acc;
          acc = OpA::apply(acc, a.parts[k]);
        }
        if (a.parts_rank > 0) excl = OpA::apply(excl, c);
        if (a.fold_res && lane == 0) *a.fold_res = acc;
      }
      if (lane == 0) gr.publish(0, ST_INCL, OpA::apply(excl, (A)agg));
    } else {
      if (!(FLAGS & SCAN_EARLY_AGG) && lane == 0) gr.publish((long)tile, ST_AGG, (A)agg);
      unsigned steps = 0, spins = 0;
      unsigned long long t1 = 0;
      if constexpr (FLAGS & SCAN_DIAG) t1 = __builtin_amdgcn_s_memrealtime();
      if constexpr (FLAGS & SCAN_NO_LOOKBACK) excl = OpA::identity(); // timing-only variant
      else excl = lookback<OP, A, LBW>(gr, (long)tile, lane, a.err, &steps, &spins);
      if constexpr (FLAGS & SCAN_DIAG) {
        if (lane == 0) {
          unsigned long long *d = a.diag + tile * 8;
          d[1] = t1;
          d[2] = __builtin_amdgcn_s_memrealtime();
          d[4] = steps;
          d[5] = spins;
          unsigned xcc;
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
          d[6] = xcc & 0xf;
        }
      }
      if (lane == 0) gr.publish((long)tile, ST_INCL, OpA::apply(excl, (A)agg));
    }
    if (lane == 0) {
      sm.s_excl = excl;
      if (tile == ntiles - 1 && a.total) *a.total = OpA::apply(excl, (A)agg);
      if (hand_next) sm.s_next = nxt;
    }
  };

  // SCAN_EARLY_AGG (commutative operators only: the thread fold is strided):
  // the tile aggregate from a fold of the registers, published before the
  // in-tile scans, so successors' look-backs find it ~1 us earlier
  C early_agg = OpC::identity();
  if constexpr ((FLAGS & SCAN_EARLY_AGG) != 0) {
    C f = OpC::identity();
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) f = OpC::apply(f, v[u][j]);
    f = wave_reduce<OP>(f);
    if (lane == 0) sm.s_early[wid] = f;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NT / kWave; w++) early_agg = OpC::apply(early_agg, sm.s_early[w]);
    if (tid == 0 && tile != 0) gr.publish((long)tile, ST_AGG, (A)early_agg);
    // SCAN_EARLY_LB: wave 0 resolves the prefix (look-back, INCL) now, while
    // the other waves run their in-tile scans; the barrier after the wave
    // scans orders s_excl before the combine
    if constexpr (FLAGS & SCAN_EARLY_LB)
      if (wid == 0) resolve(early_agg);
  }

  // ---- in-thread scan of each vector, in place
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 1; j < V; j++) v[u][j] = OpC::apply(v[u][j - 1], v[u][j]);

  // ---- U interleaved wave scans of the thread totals
  C w[U];
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = v[u][V - 1];
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = wave_inclusive_scan<OP>(w[u]);
  if (lane == kWave - 1) {
#pragma unroll
    for (int u = 0; u < U; u++) sm.s_wt[u][wid] = w[u];
  }
  // w[u] becomes the lane's exclusive prefix inside its wave
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = wave_shift_up1(w[u], OpC::identity());
  __syncthreads();

  // ---- wave 0: exclusive scan of the U x waves piece totals (flattened in
  //      element order, one piece per lane) -> s_pre; tile aggregate;
  //      publish + look-back.  The other waves hold only v and w meanwhile.
  if (wid == 0) {
    constexpr int NP = U * (NT / kWave);
    C agg = OpC::identity(); // running total of the chunks of 64 pieces
#pragma unroll
    for (int c0 = 0; c0 < NP; c0 += kWave) {
      const C pt = c0 + lane < NP ? (&sm.s_wt[0][0])[c0 + lane] : OpC::identity();
      C incl = wave_inclusive_scan<OP>(pt);
      if (c0 > 0) incl = OpC::apply(agg, incl);
      const C ex = wave_shift_up1(incl, agg); // all lanes take part in the DPP move
      if (c0 + lane < NP) (&sm.s_pre[0][0])[c0 + lane] = ex;
      agg = shfl_idx(incl, kWave - 1);
    }
    if constexpr ((FLAGS & SCAN_EARLY_AGG) != 0) agg = early_agg; // the value already published
    if constexpr (!(FLAGS & SCAN_EARLY_LB)) resolve(agg);
  }
  __syncthreads();
  const A excl = sm.s_excl;
  // fold the piece prefix into the lane prefix and the data: v = tile-local scan
#pragma unroll
  for (int u = 0; u < U; u++) {
    const C pw = OpC::apply(sm.s_pre[u][wid], w[u]);
#pragma unroll
    for (int j = 0; j < V; j++) v[u][j] = OpC::apply(pw, v[u][j]);
  }

  // ---- combine and store
  if (ALIGNED && full) {
    Vec16<T> *dst = reinterpret_cast<Vec16<T> *>(out + base);
#pragma unroll
    for (int u = 0; u < U; u++) {
      Vec16<T> r;
      if constexpr ((FLAGS & SCAN_F32_COMBINE) && std::is_same_v<C, float>) {
        const float ef = (float)excl;
#pragma unroll
        for (int j = 0; j < V; j++) r.v[j] = (T)OpC::apply(ef, v[u][j]);
      } else {
#pragma unroll
        for (int j = 0; j < V; j++) r.v[j] = (T)OpA::apply(excl, (A)v[u][j]);
      }
      if constexpr (FLAGS & SCAN_BUF_STORE) {
        u32x4 raw;
        __builtin_memcpy(&raw, &r, 16);
        __builtin_amdgcn_raw_buffer_store_b128(raw, tile_rsrc(out + base, TILE * sizeof(T)), tid * 16,
                                               u * NT * 16, (FLAGS & SCAN_NT_STORE) ? 2 /* nt */ : 0);
      } else if constexpr (FLAGS & SCAN_NT_STORE) {
        store_nt(dst + u * NT + tid, r);
      } else {
        dst[u * NT + tid] = r;
      }
    }
  } else {
    T *dst = out + base;
    const unsigned rem = (unsigned)(n - base < TILE ? n - base : TILE);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * NT + tid) * V + j;
        if (li < rem) dst[li] = (T)OpA::apply(excl, (A)v[u][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  if constexpr (FLAGS & SCAN_DIAG) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) a.diag[tile * 8 + 3] = __builtin_amdgcn_s_memrealtime();
  }
}

// One tile.  next_counter != nullptr (the persistent variant measured in
// tools/scan_sweep.hip, rejected: 2.8 ms vs 1.66 ms at 2^30 f32, because
// vmcnt also counts stores on gfx9, so a block's next loads wait for its
// previous tile's stores to drain): thread 0 claims the block's next tile
// with an atomic issued before this tile's loads and hands it over in
// s_next after the look-back.
template <int OP, typename T, bool ALIGNED, int U, int FLAGS, int NT = kScanThreads>
__device__ __forceinline__ void scan_tile(const T *in, T *out, size_t n, size_t tile, unsigned *next_counter,
                                          const granules_t<OP, T> &gr, int has_init,
                                          scan_c_t<OP, T> init, const ScanArgs<scan_acc_t<OP, T>> &a,
                                          ScanSmem<OP, T, U, NT> &sm) {
  using C = scan_c_t<OP, T>;
  using OpC = Op<OP, C>;
  constexpr int V = Vec16<T>::N;
  const int tid = threadIdx.x;
  unsigned nxt = 0;
  if (next_counter && tid == 0) nxt = atomicAdd(next_counter, 1u);

  if constexpr (FLAGS & SCAN_DIAG)
    if (tid == 0) a.diag[tile * 8 + 0] = __builtin_amdgcn_s_memrealtime();

  C v[U][V];
  scan_load<OP, T, ALIGNED, U, FLAGS, NT>(in, n, tile, v);
  if (has_init && tile == 0 && tid == 0) v[0][0] = OpC::apply(init, v[0][0]);
  scan_body<OP, T, ALIGNED, U, FLAGS, NT>(out, n, tile, v, next_counter != nullptr, nxt, gr, a, sm);
}

// One block per tile (tile index from the counter in start order).
template <int OP, typename T, bool ALIGNED, int U = kScanU, int FLAGS = kScanFlags, int MINW = kScanMinW,
          int NT = kScanThreads>
__global__ __launch_bounds__(NT, MINW) void scan_kernel(const T *in, T *out, size_t n, unsigned *counter,
                                                       granules_t<OP, T> gr, int has_init,
                                                       scan_c_t<OP, T> init, ScanArgs<scan_acc_t<OP, T>> a) {
  __shared__ ScanSmem<OP, T, U, NT> sm;
  if (threadIdx.x == 0) sm.s_tile = atomicAdd(counter, 1u);
  __syncthreads();
  scan_tile<OP, T, ALIGNED, U, FLAGS, NT>(in, out, n, sm.s_tile, nullptr, gr, has_init, init, a, sm);
}

// The tile-prefix scan (drhip_inclusive_scan_tiles), wave-part form: wave w of a
// tile owns the CONTIGUOUS part [w*Q, (w+1)*Q) of it (Q = 64*U*V elements),
// in the layout drhip_reduce_tiles reads it, and the reduce leaves every
// part's exclusive prefix (tile_local[tile*NW + w]).  So each wave scans its
// part alone: in-thread scans, U interleaved DPP wave scans, a running
// prefix over its U slot totals (read from lane 63), the given prefix, the
// stores -- no LDS, no barrier after the tile claim, no wave waiting for
// another's loads.
// Tile order of the wave-part kernel: big tiles (U >= 16) are claimed from
// a counter in start order (tile = blockIdx.x ran 1.51 vs 1.41 ms at U = 32,
// 2^30 f32: the XCDs' dispatchers drift apart), small ones (a block lives a
// few microseconds) in dispatch order.  DRHIP_WAVE_GIVEN_CLAIM = 0 / 1 forces
// one order (measurement builds).
#ifndef DRHIP_WAVE_GIVEN_CLAIM
#define DRHIP_WAVE_GIVEN_CLAIM -1
#endif
// DRHIP_WAVE_GIVEN_ORDER = 1 (measurement build): claimed tiles are taken
// from the ends of the reduce blocks' ranges first (see the claim below)
#ifndef DRHIP_WAVE_GIVEN_ORDER
#define DRHIP_WAVE_GIVEN_ORDER 0
#endif
// buffer-load cache policy of the wave-part kernel's input (2 = nt)
#ifndef DRHIP_WAVE_GIVEN_LOAD_AUX
#define DRHIP_WAVE_GIVEN_LOAD_AUX 2
#endif
template <int OP, typename T, bool ALIGNED, int U, int NT = kScanThreads>
__global__ __launch_bounds__(NT, 1) void scan_wave_given_kernel(const T *in, T *out, size_t n,
                                                              ScanArgs<scan_acc_t<OP, T>> a) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  using OpC = Op<OP, C>;
  using OpA = Op<OP, A>;
  constexpr int V = Vec16<T>::N;
  constexpr int NW = NT / kWave;
  constexpr size_t Q = (size_t)kWave * U * V; // elements per wave part
  constexpr size_t TILE = Q * NW;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  constexpr bool CLAIM = DRHIP_WAVE_GIVEN_CLAIM < 0 ? U >= 16 : DRHIP_WAVE_GIVEN_CLAIM != 0;
  size_t tile = blockIdx.x;
  if constexpr (CLAIM) {
    __shared__ unsigned s_tile;
    if (tid == 0) {
      unsigned t = atomicAdd(a.tile_counter, 1u);
      if (t == gridDim.x - 1) __hip_atomic_store(a.tile_counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if DRHIP_WAVE_GIVEN_ORDER == 1
      // tails first: claim j of reduce block b takes the block's (j+1)-th tile
      // from its END, blocks interleaved -- the tiles the step's reduce read
      // last (still in the caches) are scanned first
      {
        const unsigned per = a.tile_per, nt = gridDim.x, nb = (nt + per - 1) / per, cl = nt - (nb - 1) * per;
        unsigned b, j;
        if (t < cl * nb) {
          j = t / nb;
          b = t % nb;
        } else {
          const unsigned u = t - cl * nb;
          j = cl + u / (nb - 1);
          b = u % (nb - 1);
        }
        const unsigned len = b == nb - 1 ? cl : per;
        t = b * per + (len - 1 - j);
      }
#endif
      s_tile = t;
    }
    __syncthreads();
    tile = s_tile;
  }
  // the part's exclusive prefix: carries, then the reduce's block and part
  // prefixes -- issued ahead of the data loads
  A excl = OpA::identity();
  if (a.has_carry) excl = a.carry;
  if (a.carry_dev) excl = OpA::apply(excl, *a.carry_dev);
  if (a.parts) {
    A acc = a.parts[0], c = acc;
    for (int k = 1; k < a.parts_w; k++) {
      if (k == a.parts_rank) c = acc;
      acc = OpA::apply(acc, a.parts[k]);
    }
    if (a.parts_rank > 0) excl = OpA::apply(excl, c);
    if (tile == 0 && tid == 0 && a.fold_res) *a.fold_res = acc;
  }
  excl = OpA::apply(excl, OpA::apply(a.tile_block[tile / a.tile_per], a.tile_local[tile * NW + wid]));

  const size_t base = tile * TILE + (size_t)wid * Q;
  const bool full = base + Q <= n;
  const unsigned rem = base >= n ? 0u : (unsigned)(n - base < Q ? n - base : Q);
  C v[U][V];
  if (ALIGNED && full) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(in + base, Q * sizeof(T));
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 raw = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, u * kWave * 16, DRHIP_WAVE_GIVEN_LOAD_AUX);
      Vec16<T> r;
      __builtin_memcpy(&r, &raw, 16);
#pragma unroll
      for (int j = 0; j < V; j++) v[u][j] = (C)r.v[j];
    }
  } else {
    const T *src = in + base;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * kWave + lane) * V + j;
        v[u][j] = li < rem ? (C)src[li] : OpC::identity();
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  if (rem == 0) return; // a part past the end (the last tile's tail waves)
  // in-thread scans, then U interleaved wave scans of the thread totals
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 1; j < V; j++) v[u][j] = OpC::apply(v[u][j - 1], v[u][j]);
  C w[U];
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = wave_inclusive_scan<OP>(v[u][V - 1]);
  // slot u's prefix inside the part: the running fold of slots < u (lane
  // 63's inclusive values) and the lane's exclusive prefix in its slot
  C run = OpC::identity();
#pragma unroll
  for (int u = 0; u < U; u++) {
    const C tot = shfl_idx(w[u], kWave - 1);
    const C pw = OpC::apply(run, wave_shift_up1(w[u], OpC::identity()));
    run = OpC::apply(run, tot);
#pragma unroll
    for (int j = 0; j < V; j++) v[u][j] = OpC::apply(pw, v[u][j]);
  }
  if (ALIGNED && full) {
    Vec16<T> *dst = reinterpret_cast<Vec16<T> *>(out + base);
#pragma unroll
    for (int u = 0; u < U; u++) {
      Vec16<T> r;
#pragma unroll
      for (int j = 0; j < V; j++) r.v[j] = (T)OpA::apply(excl, (A)v[u][j]);
      store_nt(dst + u * kWave + lane, r);
    }
  } else {
    T *dst = out + base;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * kWave + lane) * V + j;
        if (li < rem) dst[li] = (T)OpA::apply(excl, (A)v[u][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
  }
}

} // namespace drhip

