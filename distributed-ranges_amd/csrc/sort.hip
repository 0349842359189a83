// sort.hip -- per-segment LSD radix sort (8-bit digits) for gfx950, plus the
// sample-sort helpers of the distributed sort.
//
// shp::sort does not exist in the reference; it is
// defined with std::ranges::sort semantics: ascending under std::less, keys
// compared as values (int32 signed, float IEEE order; -0.0 sorts before
// +0.0, which std::less calls equal).  Results are bit-identical to any
// correct sort of the same keys.
//
// One pass per 8-bit digit (4 for 4-byte keys, 8 for 8-byte keys); each pass
//   1. hist:    block b counts the digits of its chunk (CH keys, 16-B loads,
//               per-wave LDS counters) -> hist[d * nblocks + b];
//   2. scan:    inclusive scan of hist in (digit, block) order with the
//               decoupled-look-back scan kernel (scan.hip) -> off;
//   3. scatter: block b re-reads its chunk in SUB-key sub-tiles, ranks every
//               key stably (per wave: 64-lane match on the digit bits by
//               ballots, per-wave running digit counters in LDS), reorders the
//               sub-tile in LDS by digit and writes each digit's run
//               contiguously to off[d, b] - hist[d, b] + running[d].
// HBM per pass: hist reads 1x, scatter reads 1x and writes 1x (12 B/key for
// 4-byte keys; DESIGN.md "sort").  Signed and float keys are mapped to
// order-preserving unsigned bits on the first pass's load and mapped back on
// the last pass's store.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

namespace drhip {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kRadix = 256;
constexpr int kDigits1 = kRadix + 1; // + one slot for out-of-range lanes
// Two block shapes (tools/build_variant.sh + tools/sort_bench, 2^28 u32):
// small inputs 16 keys per lane x 4 sub-tiles (16 K-key chunks, 4 waves/SIMD);
// from kSortBigBytes 32 keys per lane x 8 sub-tiles (64 K-key chunks, 2
// waves/SIMD): longer digit runs per write-out and a quarter of the blocks,
// 4.19-4.25 ms vs 4.46-4.50 ms.
#ifndef DRHIP_SORT_SUBTILES
#define DRHIP_SORT_SUBTILES 4
#endif
#ifndef DRHIP_SORT_KPL4
#define DRHIP_SORT_KPL4 16
#endif
#ifndef DRHIP_SORT_MINW
#define DRHIP_SORT_MINW 4 // tools/sort_variants.sh: 4.53 vs 4.72 ms at 2^28
#endif
#ifndef DRHIP_SORT_BIG_SUBTILES
#define DRHIP_SORT_BIG_SUBTILES 8
#endif
#ifndef DRHIP_SORT_BIG_KPL4
#define DRHIP_SORT_BIG_KPL4 32
#endif
#ifndef DRHIP_SORT_BIG_MINW
#define DRHIP_SORT_BIG_MINW 2 // 3 spills (6.2-6.7 ms)
#endif
constexpr size_t kSortBigBytes = size_t(1) << 28;

template <typename K, bool BIG = false> struct SortCfg {
  static constexpr int KPL4 = BIG ? DRHIP_SORT_BIG_KPL4 : DRHIP_SORT_KPL4;
  static constexpr int SUBTILES = BIG ? DRHIP_SORT_BIG_SUBTILES : DRHIP_SORT_SUBTILES; // sub-tiles per chunk
  static constexpr int MINW = BIG ? DRHIP_SORT_BIG_MINW : DRHIP_SORT_MINW;
  static constexpr int KPL = sizeof(K) == 4 ? KPL4 : KPL4 / 2; // keys per lane per sub-tile
  static constexpr int SUB = kSortThreads * KPL;                // keys per sub-tile
  static constexpr int CH = SUB * SUBTILES;                     // keys per block chunk
  static constexpr int PASSES = (int)sizeof(K);                 // 8-bit digits
};

// onesweep sub-tile shape (one sub-tile per block): 64 keys per lane, a
// 16 K-key tile (210 VGPRs, 72 KiB LDS, 2 blocks per CU).  The look-back
// walks about (tile claim rate x status round trip) predecessors, so its
// status bytes per key fall with the square of the tile size: 2^28 u32
// 3.35 ms at 32 keys per lane (11 round trips of 4 tiles), 3.44 at 48,
// 3.04 at 64 (5.8 round trips; tools/sort_kpl.sh).
#ifndef DRHIP_SORT_OS_KPL4
#define DRHIP_SORT_OS_KPL4 64
#endif
// NT threads per block: 256 (16 K-key tiles at 64 keys per lane, 2 blocks
// per CU) or 512 (32 K-key tiles, 1 block per CU, the same 2 waves per SIMD
// and register budget): half the tiles, so half the look-back round trips
// per key and digit runs twice as long in the write-out.
template <typename K, bool BIG = true, int NT = kSortThreads> struct OsCfg {
  static constexpr int KPL4 = BIG ? DRHIP_SORT_OS_KPL4 : DRHIP_SORT_KPL4;
  // __launch_bounds__ blocks per CU: the same waves per SIMD at any NT
  static constexpr int MINW = (BIG ? DRHIP_SORT_BIG_MINW : DRHIP_SORT_MINW) * kSortThreads / NT > 0
                                  ? (BIG ? DRHIP_SORT_BIG_MINW : DRHIP_SORT_MINW) * kSortThreads / NT
                                  : 1;
  static constexpr int KPL = sizeof(K) == 4 ? KPL4 : KPL4 / 2;
  static constexpr int SUB = NT * KPL;
  static constexpr int NW = NT / kWave;
  static constexpr int PASSES = (int)sizeof(K);
};

// order-preserving key <-> unsigned bits
template <int DT> struct KeyBits;
template <> struct KeyBits<DRHIP_U32> {
  using U = uint32_t;
  __device__ static U in(U x) { return x; }
  __device__ static U out(U x) { return x; }
};
template <> struct KeyBits<DRHIP_I32> {
  using U = uint32_t;
  __device__ static U in(U x) { return x ^ 0x80000000u; }
  __device__ static U out(U x) { return x ^ 0x80000000u; }
};
template <> struct KeyBits<DRHIP_F32> {
  using U = uint32_t;
  __device__ static U in(U x) { return x ^ ((x & 0x80000000u) ? 0xFFFFFFFFu : 0x80000000u); }
  __device__ static U out(U x) { return x ^ ((x & 0x80000000u) ? 0x80000000u : 0xFFFFFFFFu); }
};
template <> struct KeyBits<DRHIP_U64> {
  using U = uint64_t;
  __device__ static U in(U x) { return x; }
  __device__ static U out(U x) { return x; }
};
template <> struct KeyBits<DRHIP_I64> {
  using U = uint64_t;
  __device__ static U in(U x) { return x ^ 0x8000000000000000ull; }
  __device__ static U out(U x) { return x ^ 0x8000000000000000ull; }
};
template <> struct KeyBits<DRHIP_F64> {
  using U = uint64_t;
  __device__ static U in(U x) {
    return x ^ ((x & 0x8000000000000000ull) ? ~0ull : 0x8000000000000000ull);
  }
  __device__ static U out(U x) {
    return x ^ ((x & 0x8000000000000000ull) ? 0x8000000000000000ull : ~0ull);
  }
};

// ---------------------------------------------------------------- hist
template <int DT, bool XIN, bool BIG>
__global__ __launch_bounds__(kSortThreads) void radix_hist(const typename KeyBits<DT>::U *keys, size_t n,
                                                          int shift, uint32_t *hist, unsigned nblocks,
                                                          bool aligned) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U, BIG>;
  constexpr int V = 16 / sizeof(U);
  __shared__ uint32_t s_cnt[kSortWaves][kRadix];
  const int tid = threadIdx.x, wid = tid / kWave;
  for (int i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * Cfg::CH;
  const size_t end = base + Cfg::CH < n ? base + Cfg::CH : n;
  const Vec16<U> *kv = reinterpret_cast<const Vec16<U> *>(keys);
  if (aligned && end - base == (size_t)Cfg::CH) {
    // full chunk of a 16-byte aligned array: CH / V vectors, strided by the block
#pragma unroll 4
    for (int i = tid; i < Cfg::CH / V; i += kSortThreads) {
      const Vec16<U> x = load_nt(kv + base / V + i);
#pragma unroll
      for (int j = 0; j < V; j++) {
        const U k = XIN ? KeyBits<DT>::in(x.v[j]) : x.v[j];
        atomicAdd(&s_cnt[wid][(unsigned)(k >> shift) & 0xFF], 1u);
      }
    }
  } else {
    for (size_t i = base + tid; i < end; i += kSortThreads) {
      const U k = XIN ? KeyBits<DT>::in(keys[i]) : keys[i];
      atomicAdd(&s_cnt[wid][(unsigned)(k >> shift) & 0xFF], 1u);
    }
  }
  __syncthreads();
  for (int d = tid; d < kRadix; d += kSortThreads) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kSortWaves; w++) t += s_cnt[w][d];
    hist[(size_t)d * nblocks + blockIdx.x] = t;
  }
}

// ------------------------------------------------- sub-tile ranking
// Shared by the classic scatter and the onesweep kernel: one sub-tile of
// SUB keys (KPL per lane, wave w owning the contiguous keys [w*KPW,
// (w+1)*KPW)) is ranked stably, counted per digit and reordered by digit in
// LDS.
template <typename U, int SUB, int NW = kSortWaves> struct RankSmem {
  U keys[SUB];
  uint32_t wcnt[NW][kDigits1];   // per-wave running counts / prefixes
  uint32_t start[kDigits1];      // digit start inside the sub-tile
  uint32_t sub[kDigits1];        // sub-tile digit totals
  uint32_t wsum[kRadix / kWave]; // the digit scan's wave totals
};

// stable rank inside the wave's contiguous run of keys: the lanes holding the
// same digit (peers) are the AND over the digit's bits of (bit set ? ballot :
// ~ballot), kept as two 32-bit halves so each bit costs one compare and two
// 3-input bit ops (x & ~(sign ^ ballot)); the 9th bit (out-of-range slot)
// only on the partial last sub-tile.  Leaves two 16-bit ranks per register
// in rank2 and the wave's digit counts in sm.wcnt[wid].
template <typename U, int KPL, int KPW, int NB>
__device__ __forceinline__ void rank_keys(const U (&key)[KPL], uint32_t (&rank2)[(KPL + 1) / 2], unsigned valid,
                                          int shift, uint32_t (&wcnt)[kDigits1], int lane, int wid) {
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t lt_lo = (uint32_t)lt_mask, lt_hi = (uint32_t)(lt_mask >> 32);
#pragma unroll
  for (int r = 0; r < KPL; r++) {
    const unsigned li = wid * KPW + r * kWave + lane;
    const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
    uint32_t plo = ~0u, phi = ~0u;
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const uint32_t sgn = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1); // 0 or ~0
      const uint64_t m = __ballot(sgn != 0u);
      // peers &= ~(sgn ^ ballot): one v_bitop3 per half (LUT 0x90 with
      // src0/1/2 = 0xf0/0xcc/0xaa), the ballot half read as an SGPR; the
      // s_nop covers the VALU-writes-SGPR -> VALU-reads-it hazard the
      // compiler cannot see through inline asm
      asm volatile("s_nop 1\n\tv_bitop3_b32 %0, %2, %3, %4 bitop3:0x90\n\tv_bitop3_b32 %1, %5, %3, %6 bitop3:0x90"
                   : "=&v"(plo), "=&v"(phi)
                   : "v"(plo), "v"(sgn), "s"((uint32_t)m), "v"(phi), "s"((uint32_t)(m >> 32)));
    }
    const uint32_t before = wcnt[d];
    const unsigned below = (unsigned)(__builtin_popcount(plo & lt_lo) + __builtin_popcount(phi & lt_hi));
    const uint32_t rk = before + below;
    if (r & 1) rank2[r / 2] |= rk << 16;
    else rank2[r / 2] = rk;
    // the lowest lane of each peer group advances the wave's counter
    if (below == 0) wcnt[d] = before + (uint32_t)(__builtin_popcount(plo) + __builtin_popcount(phi));
  }
}

// The same ranking with ONE LDS atomic per key: ds_add_rtn_u32 on the wave's
// counter of the key's digit returns the count so far, and the lanes of one
// wave-instruction that hit the same counter get their old values in
// ascending lane order (measured: tools/lds_atomic_order, 0 of 9.6e8
// same-address lane pairs out of order; checked again on every device before
// the first sort uses it, sort_rank_atomic below), so slot-by-slot issue
// gives the stable rank.  Replaces 8 ballots + 16 bit-ops + a counter read
// and write per key.
// DRHIP_SORT_UNI_FAST = 1: a wave whose keys all share the digit being
// ranked or counted takes ONE LDS update instead of 64 same-address atomics
// per round (skewed keys: tools/r06/sort_skew_probe.py)
#ifndef DRHIP_SORT_UNI_FAST
#define DRHIP_SORT_UNI_FAST 1
#endif
constexpr bool kSortUniFast = DRHIP_SORT_UNI_FAST;
// DRHIP_SORT_UNI_NXT = 1: the same for the next-digit count of the
// persistent onesweep's write-out (one check per round of every wave)
#ifndef DRHIP_SORT_UNI_NXT
#define DRHIP_SORT_UNI_NXT 0
#endif
constexpr bool kSortUniNxt = DRHIP_SORT_UNI_NXT;
// DRHIP_SORT_FEW_K = K > 0 (measurement knob, default 0): a wave whose first
// round holds at most K distinct digits (the exponent byte of floats: a few
// values per wave) ranks / counts those digits with ballots into K
// wave-uniform counters -- no LDS atomic, whose same-address lanes would
// serialise -- and only the other digits' keys with atomics.  K = 4: f32
// U[0,1) keys 3.66 -> 3.16 ms at 2^28, but uniform keys 3 % slower (the
// per-tile probe), so it stays off (profiles/r06x_sort_few_ab.txt).
#ifndef DRHIP_SORT_FEW_K
#define DRHIP_SORT_FEW_K 0
#endif
constexpr int kSortFewK = DRHIP_SORT_FEW_K;
constexpr int kFewN = kSortFewK > 0 ? kSortFewK : 1; // array extent
// DRHIP_SORT_FEW_HIST = 1: the same for the pre-pass counts (a per-tile probe
// of every position; no histogram is known yet)
#ifndef DRHIP_SORT_FEW_HIST
#define DRHIP_SORT_FEW_HIST 0
#endif
constexpr bool kSortFewHist = DRHIP_SORT_FEW_HIST;

// The first distinct values of v over the wave's lanes, in lane order, into
// c[0..K) (wave-uniform); returns how many (K + 1: more than K exist).
template <int K> __device__ __forceinline__ int wave_distinct(unsigned v, unsigned (&c)[K]) {
  uint64_t todo = __ballot(1);
  int n = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    c[k] = 0xFFFFFFFFu; // matches no digit
    if (todo) {
      const int l0 = __builtin_ctzll(todo);
      const unsigned dl = __builtin_amdgcn_readlane(v, l0);
      c[k] = dl;
      n = k + 1;
      todo &= ~__ballot(v == dl);
    }
  }
  return todo ? K + 1 : n;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

template <typename U, int KPL, int KPW>
__device__ __forceinline__ void rank_keys_atomic(const U (&key)[KPL], uint32_t (&rank2)[(KPL + 1) / 2],
                                                 unsigned valid, int shift, uint32_t (&wcnt)[kDigits1], int lane,
                                                 int wid, bool few_ok = true) {
  if constexpr (kSortUniFast) {
    // every key of this wave valid and of ONE digit (small integers' high
    // bytes, constant fields): the atomic path would serialise 64 lanes on
    // one LDS counter per round; the ranks it returns are r * 64 + lane
    // first round only (3 instructions for keys that differ), then the rest
    const unsigned d0 = (unsigned)(key[0] >> shift) & 0xFF;
    const unsigned dw = __builtin_amdgcn_readfirstlane(d0);
    bool same = wid * KPW + (KPL - 1) * kWave + kWave <= valid;
    if (__all(same && d0 == dw)) {
#pragma unroll
      for (int r = 1; r < KPL; r++) same = same && ((unsigned)(key[r] >> shift) & 0xFF) == dw;
    } else {
      same = false;
    }
    if (__all(same)) {
      if (lane == 0) wcnt[dw] += (uint32_t)(KPL * kWave);
#pragma unroll
      for (int r = 0; r < KPL; r++) {
        const uint32_t rk = (uint32_t)(r * kWave + lane);
        if (r & 1) rank2[r / 2] |= rk << 16;
        else rank2[r / 2] = rk;
      }
      return;
    }
  }
  if constexpr (kSortFewK > 0) {
    // at most kSortFewK distinct digits in the first round: those digits get
    // their ranks from ballots (rank = the digit's count in earlier rounds +
    // its lanes below this one: the atomics' order), any other digit from
    // the atomics; each digit takes one of the two ways for the whole tile
    unsigned cand[kFewN];
    const unsigned dr0 = wid * KPW + lane < valid ? (unsigned)(key[0] >> shift) & 0xFF : (unsigned)kRadix;
    const int nd = few_ok ? wave_distinct<kFewN>(dr0, cand) : kSortFewK + 1;
    if (nd <= kSortFewK) {
      uint32_t run[kFewN];
#pragma unroll
      for (int k = 0; k < kSortFewK; k++) run[k] = 0;
#pragma unroll
      for (int r = 0; r < KPL; r++) {
        const unsigned li = wid * KPW + r * kWave + lane;
        const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
        uint32_t rk = 0;
        bool hit = false;
#pragma unroll
        for (int k = 0; k < kSortFewK; k++) {
          const uint64_t m = __ballot(d == cand[k]);
          if (d == cand[k]) {
            rk = run[k] + lanes_below(m);
            hit = true;
          }
          run[k] += (uint32_t)__builtin_popcountll(m);
        }
        if (!hit) rk = atomicAdd(&wcnt[d], 1u);
        if (r & 1) rank2[r / 2] |= rk << 16;
        else rank2[r / 2] = rk;
        __builtin_amdgcn_sched_barrier(0); // one round's ballots live at a time
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kSortFewK; k++)
          if (k < nd) wcnt[cand[k]] += run[k];
      }
      return;
    }
  }
#pragma unroll
  for (int r = 0; r < KPL; r++) {
    const unsigned li = wid * KPW + r * kWave + lane;
    const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
    const uint32_t rk = atomicAdd(&wcnt[d], 1u);
    if (r & 1) rank2[r / 2] |= rk << 16;
    else rank2[r / 2] = rk;
  }
}

template <bool AR, typename U, int KPL, int KPW>
__device__ __forceinline__ void rank_subtile(const U (&key)[KPL], uint32_t (&rank2)[(KPL + 1) / 2], unsigned valid,
                                             unsigned full, int shift, uint32_t (&wcnt)[kDigits1], int lane, int wid,
                                             bool few_ok = true) {
  if constexpr (AR) {
    rank_keys_atomic<U, KPL, KPW>(key, rank2, valid, shift, wcnt, lane, wid, few_ok);
  } else {
    if (valid == full) rank_keys<U, KPL, KPW, 8>(key, rank2, valid, shift, wcnt, lane, wid);
    else rank_keys<U, KPL, KPW, 9>(key, rank2, valid, shift, wcnt, lane, wid);
  }
}

// After ranking and a barrier: the sub-tile total of every digit (sm.sub),
// the digit's start inside the sub-tile (sm.start, exclusive scan of sm.sub
// over 257 entries) and, in sm.wcnt[w][d], the LDS slot of wave w's first
// key of digit d (start + the counts of the waves before w), so the reorder
// reads one table entry per key.  Ends with a barrier.
template <typename U, int SUB, int NW>
__device__ __forceinline__ void digit_offsets(RankSmem<U, SUB, NW> &sm, int tid) {
  constexpr int NT = NW * kWave;
  const int lane = tid & (kWave - 1), wid = tid / kWave;
  for (int d = tid; d < kDigits1; d += NT) {
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) run += sm.wcnt[w][d];
    sm.sub[d] = run;
  }
  __syncthreads();
  // thread t < 256 scans entry t with a DPP wave scan + LDS wave totals;
  // entry 256 last.
  const uint32_t x = tid < kRadix ? sm.sub[tid] : 0u;
  const uint32_t incl = wave_inclusive_scan<DRHIP_PLUS>(x);
  if (tid < kRadix && lane == kWave - 1) sm.wsum[wid] = incl;
  __syncthreads();
  if (tid < kRadix) {
    uint32_t wpre = 0;
#pragma unroll
    for (int w = 0; w < kRadix / kWave; w++) wpre += w < wid ? sm.wsum[w] : 0u;
    const uint32_t st = wpre + incl - x;
    sm.start[tid] = st;
    {
      uint32_t run = st;
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t c = sm.wcnt[w][tid];
        sm.wcnt[w][tid] = run;
        run += c;
      }
    }
    if (tid == kRadix - 1) {
      const uint32_t st1 = wpre + incl;
      sm.start[kRadix] = st1;
      uint32_t run = st1;
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t c = sm.wcnt[w][kRadix];
        sm.wcnt[w][kRadix] = run;
        run += c;
      }
    }
  }
  __syncthreads();
}

// reorder the ranked sub-tile by digit into sm.keys (valid keys land in
// [0, valid)); needs a barrier before sm.keys is read.
template <typename U, int SUB, int KPL, int KPW, int NW = kSortWaves>
__device__ __forceinline__ void reorder_keys(RankSmem<U, SUB, NW> &sm, const U (&key)[KPL],
                                             const uint32_t (&rank2)[(KPL + 1) / 2], unsigned valid, int shift,
                                             int lane, int wid) {
#pragma unroll
  for (int r = 0; r < KPL; r++) {
    const unsigned li = wid * KPW + r * kWave + lane;
    const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
    const uint32_t rk = (r & 1) ? rank2[r / 2] >> 16 : rank2[r / 2] & 0xFFFFu;
    sm.keys[sm.wcnt[wid][d] + rk] = key[r];
  }
}

// load sub-tile keys: round r covers w*KPW + r*64 + lane (coalesced)
template <int DT, bool XIN, int KPL, int KPW>
__device__ __forceinline__ void load_subtile(typename KeyBits<DT>::U (&key)[KPL], const typename KeyBits<DT>::U *src,
                                             size_t sb, unsigned vld, int lane, int wid) {
  using U = typename KeyBits<DT>::U;
#pragma unroll
  for (int r = 0; r < KPL; r++) {
    const unsigned li = wid * KPW + r * kWave + lane;
    U k = li < vld ? __builtin_nontemporal_load(src + sb + li) : U(0);
    if (XIN) k = KeyBits<DT>::in(k);
    key[r] = k;
  }
}

// -------------------------------------------------------------- scatter
template <int DT, bool XIN, bool XOUT, bool BIG, bool AR>
__global__ __launch_bounds__(kSortThreads, (SortCfg<typename KeyBits<DT>::U, BIG>::MINW)) void radix_scatter(
    const typename KeyBits<DT>::U *src, typename KeyBits<DT>::U *dst, size_t n, int shift, const uint32_t *hist,
    const uint32_t *off, unsigned nblocks) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U, BIG>;
  constexpr int kSubTiles = Cfg::SUBTILES;
  constexpr int KPL = Cfg::KPL;
  constexpr int SUB = Cfg::SUB;
  constexpr int KPW = SUB / kSortWaves; // keys per wave per sub-tile (contiguous)

  __shared__ RankSmem<U, SUB> sm;
  __shared__ uint32_t s_run[kRadix]; // global write cursor per digit
  __shared__ uint32_t s_cur[kRadix]; // s_run - the digit's start in the sub-tile

  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const size_t base = (size_t)blockIdx.x * Cfg::CH;
  for (int d = tid; d < kRadix; d += kSortThreads) {
    const size_t h = (size_t)d * nblocks + blockIdx.x;
    s_run[d] = off[h] - hist[h];
  }
  for (int i = tid; i < kSortWaves * kDigits1; i += kSortThreads) (&sm.wcnt[0][0])[i] = 0;
  __syncthreads();

  // The next sub-tile is loaded as soon as this one's keys are in LDS, so its
  // latency hides under the write-out phase.
  U key[KPL];
  auto valid_at = [&](size_t sb) -> unsigned {
    return sb < n ? (unsigned)(n - sb < (size_t)SUB ? n - sb : (size_t)SUB) : 0u;
  };
  size_t sbase = base;
  unsigned valid = valid_at(sbase);
  if (valid) load_subtile<DT, XIN, KPL, KPW>(key, src, sbase, valid, lane, wid);
  for (int st = 0; st < kSubTiles; st++) {
    if (!valid) break; // uniform
    uint32_t rank2[(KPL + 1) / 2]; // two 16-bit ranks per register (no spills at 4 waves/SIMD)
    rank_subtile<AR, U, KPL, KPW>(key, rank2, valid, (unsigned)SUB, shift, sm.wcnt[wid], lane, wid);
    __syncthreads();
    digit_offsets(sm, tid);
    reorder_keys<U, SUB, KPL, KPW>(sm, key, rank2, valid, shift, lane, wid);
    // global cursor of digit d minus its start in the sub-tile: key p of the
    // reordered sub-tile goes to s_cur[d] + p
    for (int d = tid; d < kRadix; d += kSortThreads) s_cur[d] = s_run[d] - sm.start[d];
    const size_t nbase = sbase + SUB;
    const unsigned nvalid = st + 1 < kSubTiles ? valid_at(nbase) : 0u;
    if (nvalid) load_subtile<DT, XIN, KPL, KPW>(key, src, nbase, nvalid, lane, wid);
    __syncthreads();
    // ---- write each digit's run contiguously (valid keys occupy [0, valid))
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned p = r * kSortThreads + tid;
      if (p < valid) {
        const U k = sm.keys[p];
        const unsigned d = (unsigned)(k >> shift) & 0xFF;
        dst[s_cur[d] + p] = XOUT ? KeyBits<DT>::out(k) : k;
      }
    }
    __syncthreads();
    for (int d = tid; d < kRadix; d += kSortThreads) s_run[d] += sm.sub[d];
    for (int i = tid; i < kSortWaves * kDigits1; i += kSortThreads) (&sm.wcnt[0][0])[i] = 0;
    __syncthreads();
    sbase = nbase;
    valid = nvalid;
  }
}

// ------------------------------------------------------------ onesweep
// One histogram pass for every digit position, then one kernel per pass
// that ranks a sub-tile, publishes its digit counts and finds the counts of
// all earlier sub-tiles by decoupled look-back (Merrill & Garland's
// single-pass prefix scan applied per digit, as in Adinets & Merrill's
// "Onesweep"), so no per-pass histogram re-read of the keys: 4 B/key once +
// 8 B/key per pass (36 B/key for 4-byte keys instead of 48).
//
// Status: one 8-B word per (sub-tile, digit) = count | (epoch << 2 | flag)
// << 32, written by ONE agent-scope 8-B atomic store and read by one 8-B
// agent-scope load, so count and flag cannot be seen apart.  The words are
// zeroed once per sort; pass p uses epoch p + 1, so a word from an earlier
// pass reads as "not yet published".
constexpr unsigned kOsAgg = 1, kOsIncl = 2;
#ifndef DRHIP_SORT_OS_LOOK
#define DRHIP_SORT_OS_LOOK 4
#endif
constexpr int kOsLook = DRHIP_SORT_OS_LOOK; // predecessors read per look-back round trip
#ifndef DRHIP_SORT_CNT_WO
#define DRHIP_SORT_CNT_WO 1
#endif
constexpr unsigned kOsSpinLimit = 1u << 22;

// ---- onesweep pass-0 bases without a look-back ------------------------
// Pass 0 reads the keys in input order, so its per-tile digit counts can be
// taken before it runs: radix_tile_hist0 counts digit position 0 of every
// onesweep tile (tilecnt[tile][d], plus chunk totals over kOsChunk tiles)
// and positions 1.. for the whole range (kH0All; position 1 only with
// DRHIP_SORT_H0_ALL=0, positions 2.. then counted by passes 1.. during their
// write-out); radix_chunk_bases scans the chunk totals per digit,
// radix_tile_bases rewrites tilecnt into each tile's output base per digit.
// DRHIP_SORT_H0_CNT1 = 1 (default): radix_tile_hist0 also counts digit
// position 1 (2 LDS atomics per key in the pre-pass); 0: pass 0 counts it
// during its write-out like the middle passes, so the pre-pass makes one
// LDS atomic per key (measured slower: pass 0 spills, DESIGN.md sort notes)
#ifndef DRHIP_SORT_H0_CNT1
#define DRHIP_SORT_H0_CNT1 1
#endif
constexpr bool kH0Cnt1 = DRHIP_SORT_H0_CNT1;
// DRHIP_SORT_H0_ALL = 1 (default, round 6): radix_tile_hist0 counts EVERY
// position >= 1 (one LDS atomic per key and position in the pre-pass, or one
// add per wave where the wave's keys share the digit), so no onesweep pass
// counts a next digit under its scattered write-out.  Uniform u32 keys: the
// same time as counting in the passes (profiles/r06_sort_h0all_ab.txt);
// skewed keys (small integers, constant high bytes): with the wave-uniform
// fast paths 2.72-2.85 ms at 2^28 instead of 4.1-8.65 ms
// (profiles/r06t_sort_skew_ab.txt).
#ifndef DRHIP_SORT_H0_ALL
#define DRHIP_SORT_H0_ALL 1
#endif
constexpr bool kH0All = DRHIP_SORT_H0_ALL;
constexpr int kOsChunk = 64;     // tiles per chunk of the tile scan
constexpr int kOsHistParts = 64; // partial histograms per digit position (atomic spread)

template <int DT, bool BIG, int NT = kSortThreads>
__global__ __launch_bounds__(NT) void radix_tile_hist0(const typename KeyBits<DT>::U *keys, size_t n,
                                                      uint32_t *tilecnt, uint32_t *chunksum, uint32_t *parts1) {
  using U = typename KeyBits<DT>::U;
  using Cfg = OsCfg<U, BIG, NT>;
  constexpr int NW = Cfg::NW;
  constexpr int KPL = Cfg::KPL, SUB = Cfg::SUB, KPW = SUB / NW;
  constexpr int V = 16 / sizeof(U), NV = SUB / V / NT; // 16-byte vectors per lane
  // positions counted here: 0 per tile, 1 (kH0Cnt1) or all (kH0All) globally
  constexpr int NPOS = kH0All ? (int)sizeof(U) : 2;
  __shared__ uint32_t s_cnt[NPOS][NW][kRadix];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  for (int i = tid; i < NPOS * NW * kRadix; i += NT) (&s_cnt[0][0][0])[i] = 0;
  const size_t sbase = (size_t)blockIdx.x * SUB;
  const unsigned valid = (unsigned)(n - sbase < (size_t)SUB ? n - sbase : (size_t)SUB);
  constexpr int NCNT = (kH0All || kH0Cnt1) ? NPOS : 1; // positions counted
  // uni: bit p set when position p was counted for the whole wave at once
  auto count = [&](U k, unsigned uni) {
    k = KeyBits<DT>::in(k);
#pragma unroll
    for (int p = 0; p < NCNT; p++)
      if (!(uni >> p & 1u)) atomicAdd(&s_cnt[p][wid][(unsigned)(k >> (8 * p)) & 0xFF], 1u);
  };
  if (((uintptr_t)(keys + sbase) & 15) == 0) {
    // 16-byte nontemporal vectors, all issued before any count
    const Vec16<U> *kv = reinterpret_cast<const Vec16<U> *>(keys + sbase);
    Vec16<U> x[NV];
#pragma unroll
    for (int r = 0; r < NV; r++) {
      const unsigned vi = r * NT + tid;
      if ((vi + 1) * V <= valid) x[r] = load_nt(kv + vi);
    }
    __syncthreads();
    unsigned uni = 0;
    if constexpr (kSortUniFast) {
      // a full tile whose wave holds ONE digit at position p: one LDS add for
      // the wave's NV * V * 64 keys instead of 64 same-address atomics per key
      if (valid == (unsigned)SUB) {
#pragma unroll
        for (int p = 0; p < NCNT; p++) {
          // the first key of every lane first (3 instructions for keys that
          // differ), then the rest
          const unsigned d0 = (unsigned)(KeyBits<DT>::in(x[0].v[0]) >> (8 * p)) & 0xFF;
          const unsigned dw = __builtin_amdgcn_readfirstlane(d0);
          bool same = false;
          if (__all(d0 == dw)) {
            same = true;
#pragma unroll
            for (int r = 0; r < NV; r++)
#pragma unroll
              for (int j = 0; j < V; j++) same = same && ((unsigned)(KeyBits<DT>::in(x[r].v[j]) >> (8 * p)) & 0xFF) == dw;
          }
          if (__all(same)) {
            uni |= 1u << p;
            if (lane == 0) s_cnt[p][wid][dw] += (uint32_t)(NV * V * kWave);
          }
        }
      }
    }
    // positions whose first keys show at most kSortFewK digits across the
    // wave: ballot counts into wave-uniform counters, atomics only for the
    // other digits (full tiles)
    unsigned few = 0;
    unsigned cand[NCNT][kFewN];
    uint32_t run[NCNT][kFewN];
    if constexpr (kSortFewK > 0 && kSortFewHist) {
      if (valid == (unsigned)SUB) {
#pragma unroll
        for (int p = 0; p < NCNT; p++) {
#pragma unroll
          for (int k = 0; k < kSortFewK; k++) run[p][k] = 0;
          if (!(uni >> p & 1u)) {
            const unsigned d0 = (unsigned)(KeyBits<DT>::in(x[0].v[0]) >> (8 * p)) & 0xFF;
            if (wave_distinct<kFewN>(d0, cand[p]) <= kSortFewK) few |= 1u << p;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < NV; r++) {
      const unsigned vi = r * NT + tid;
      if ((vi + 1) * V <= valid) {
#pragma unroll
        for (int j = 0; j < V; j++) {
          if constexpr (kSortFewK > 0 && kSortFewHist) {
            if (few) {
              const U k = KeyBits<DT>::in(x[r].v[j]);
#pragma unroll
              for (int p = 0; p < NCNT; p++) {
                if (uni >> p & 1u) continue;
                const unsigned dp = (unsigned)(k >> (8 * p)) & 0xFF;
                if (few >> p & 1u) {
                  bool hit = false;
#pragma unroll
                  for (int c = 0; c < kSortFewK; c++) {
                    const uint64_t m = __ballot(dp == cand[p][c]);
                    hit = hit || dp == cand[p][c];
                    run[p][c] += (uint32_t)__builtin_popcountll(m);
                  }
                  if (!hit) atomicAdd(&s_cnt[p][wid][dp], 1u);
                } else {
                  atomicAdd(&s_cnt[p][wid][dp], 1u);
                }
              }
              __builtin_amdgcn_sched_barrier(0);
              continue;
            }
          }
          count(x[r].v[j], uni);
        }
      } else {
        for (unsigned e = vi * V; e < valid && e < (vi + 1) * V; e++) count(keys[sbase + e], 0u);
      }
    }
    if constexpr (kSortFewK > 0 && kSortFewHist) {
      if (few && lane == 0) {
#pragma unroll
        for (int p = 0; p < NCNT; p++)
          if (few >> p & 1u) {
#pragma unroll
            for (int c = 0; c < kSortFewK; c++)
              if (cand[p][c] < (unsigned)kRadix) s_cnt[p][wid][cand[p][c]] += run[p][c];
          }
      }
    }
  } else {
    U key[KPL];
    load_subtile<DT, false, KPL, KPW>(key, keys, sbase, valid, lane, wid);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KPL; r++)
      if (wid * KPW + r * kWave + lane < valid) count(key[r], 0u);
  }
  __syncthreads();
  const int d = tid;
  if (d >= kRadix) return;
  uint32_t c0 = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) c0 += s_cnt[0][w][d];
  tilecnt[(size_t)blockIdx.x * kRadix + d] = c0;
  if (c0) atomicAdd(chunksum + (size_t)(blockIdx.x / kOsChunk) * kRadix + d, c0);
  if constexpr (kH0All || kH0Cnt1) {
    // position p's partials at parts1 + (p - 1) * kOsHistParts * kRadix
#pragma unroll
    for (int p = 1; p < NPOS; p++) {
      uint32_t c = 0;
#pragma unroll
      for (int w = 0; w < NW; w++) c += s_cnt[p][w][d];
      if (c) atomicAdd(parts1 + ((size_t)(p - 1) * kOsHistParts + blockIdx.x % kOsHistParts) * kRadix + d, c);
    }
  }
}

// block d, thread c: exclusive scan of digit d's chunk totals over the
// chunks (in place); digit d's total to tot[d]
__global__ __launch_bounds__(kSortThreads) void radix_chunk_bases(uint32_t *chunksum, unsigned nchunks,
                                                                 uint32_t *tot) {
  __shared__ uint32_t s_w[kSortWaves];
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const unsigned per = (nchunks + kSortThreads - 1) / kSortThreads; // consecutive chunks per thread
  const unsigned c0 = tid * per, c1 = c0 + per < nchunks ? c0 + per : nchunks;
  uint32_t sum = 0;
  for (unsigned c = c0; c < c1; c++) sum += chunksum[(size_t)c * kRadix + d];
  const uint32_t incl = wave_inclusive_scan<DRHIP_PLUS>(sum);
  if (lane == kWave - 1) s_w[wid] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
#pragma unroll
  for (int w = 0; w < kSortWaves; w++) run += w < wid ? s_w[w] : 0u;
  if (tid == kSortThreads - 1) tot[d] = run + sum;
  for (unsigned c = c0; c < c1; c++) {
    const uint32_t v = chunksum[(size_t)c * kRadix + d];
    chunksum[(size_t)c * kRadix + d] = run;
    run += v;
  }
}

// block c, thread d: tilecnt[t][d] <- output base of digit d in tile t
// (digit start + chunk base + the tiles before t in the chunk)
__global__ __launch_bounds__(kRadix) void radix_tile_bases(uint32_t *tilecnt, const uint32_t *chunksum,
                                                          const uint32_t *dstart, size_t tiles) {
  const int d = threadIdx.x;
  const size_t t0 = (size_t)blockIdx.x * kOsChunk;
  uint32_t run = dstart[d] + chunksum[(size_t)blockIdx.x * kRadix + d];
  uint32_t v[kOsChunk];
#pragma unroll
  for (int i = 0; i < kOsChunk; i++) v[i] = t0 + i < tiles ? tilecnt[(t0 + i) * kRadix + d] : 0u;
#pragma unroll
  for (int i = 0; i < kOsChunk; i++) {
    if (t0 + i < tiles) tilecnt[(t0 + i) * kRadix + d] = run;
    run += v[i];
  }
}

// dstart[d] of one digit position from its kOsHistParts partial histograms
__global__ __launch_bounds__(kRadix) void radix_digit_starts_parts(const uint32_t *parts, uint32_t *dstart) {
  __shared__ uint32_t s_w[kRadix / kWave];
  const int d = threadIdx.x, lane = d & (kWave - 1), wid = d / kWave;
  uint32_t x = 0;
#pragma unroll 8
  for (int j = 0; j < kOsHistParts; j++) x += parts[j * kRadix + d];
  const uint32_t incl = wave_inclusive_scan<DRHIP_PLUS>(x);
  if (lane == kWave - 1) s_w[wid] = incl;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (int w = 0; w < kRadix / kWave; w++) pre += w < wid ? s_w[w] : 0u;
  dstart[d] = pre + incl - x;
}

// Diagnostic build only (-DDRHIP_SORT_STAMPS, tools/sort_stamps.sh): per
// tile of the pass with epoch DRHIP_SORT_STAMP_EPOCH, thread 0 records the
// real-time clock at block start and end and shader-clock phase marks, plus
// its look-back round trips; read back by drhip_dbg_sort_stamps.
#ifdef DRHIP_SORT_STAMPS
#ifndef DRHIP_SORT_STAMP_EPOCH
#define DRHIP_SORT_STAMP_EPOCH 2
#endif
constexpr int kStampSlots = 10;
constexpr size_t kStampTiles = 1 << 16;
__device__ unsigned long long g_sort_stamps[kStampTiles * kStampSlots];
__device__ __forceinline__ unsigned long long stamp_clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long stamp_rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define OS_STAMP(k, v)                                                                 \
  do {                                                                                 \
    if (stamp_on) st_v[k] = (v);                                                       \
  } while (0)
#else
#define OS_STAMP(k, v) \
  do {                 \
  } while (0)
#endif

// 4-byte status words (W32, segments of < 2^30 keys): flag in bits 31:30
// (AGG / INCL), count or inclusive prefix in bits 29:0 -- half the bytes of
// every publish and look-back read.  Without an epoch field, passes
// alternate between two word arrays and each tile zeroes its row of the
// array the NEXT pass uses (the pass before it has finished), so only array
// 0 needs a memset per sort.
//
// Pass 0 (XIN) takes every tile's digit bases from `pre` (radix_tile_hist0 +
// the tile scan below: the input order is known before the pass), so it has
// no look-back and publishes nothing.  Every pass but the last counts the
// NEXT digit position of its keys in the look-back's shadow (per-wave LDS
// counters, then one atomic per digit into one of kOsHistParts partial
// histograms), so no pass re-reads the keys for a histogram.
template <int DT, bool XIN, bool XOUT, bool BIG, bool AR, bool W32>
__global__ __launch_bounds__(kSortThreads, (OsCfg<typename KeyBits<DT>::U, BIG>::MINW)) void radix_onesweep(
    const typename KeyBits<DT>::U *src, typename KeyBits<DT>::U *dst, size_t n, int shift, const uint32_t *dstart,
    const uint32_t *pre, void *status_v, uint32_t *status_next, uint32_t *nxt_hist, unsigned *counter,
    unsigned epoch, unsigned *err) {
  using U = typename KeyBits<DT>::U;
  using Cfg = OsCfg<U, BIG>;
  constexpr int KPL = Cfg::KPL;
  constexpr int SUB = Cfg::SUB;
  constexpr int KPW = SUB / kSortWaves;
  // middle passes count the next digit position (pass 0's next position is
  // counted by radix_tile_hist0)
  constexpr bool NXT = !XOUT && !(XIN && kH0Cnt1) && !kH0All;

  __shared__ RankSmem<U, SUB> sm;
  __shared__ uint32_t s_run[kRadix];
  __shared__ uint32_t s_nxt[NXT ? kSortWaves : 1][kRadix];
  __shared__ unsigned s_tile;

  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
#ifdef DRHIP_SORT_STAMPS
  const bool stamp_on = tid == 0 && epoch == DRHIP_SORT_STAMP_EPOCH;
  unsigned long long st_v[kStampSlots] = {};
  unsigned trips = 0, waits = 0; // round trips; those that found an unpublished predecessor
  OS_STAMP(0, stamp_rt());
  OS_STAMP(1, stamp_clk());
#endif
  // tiles are claimed in start order, so every look-back waits only on
  // blocks that are already running (no dependence on dispatch order)
  if (XIN) {
    if (tid == 0) s_tile = blockIdx.x; // no look-back: any order
  } else if (tid == 0) {
    s_tile = atomicAdd(counter, 1u);
  }
  for (int i = tid; i < kSortWaves * kDigits1; i += kSortThreads) (&sm.wcnt[0][0])[i] = 0;
  if constexpr (NXT)
    for (int i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&s_nxt[0][0])[i] = 0;
  __syncthreads();
  const unsigned tile = s_tile;
  const size_t sbase = (size_t)tile * SUB;
  const unsigned valid = (unsigned)(n - sbase < (size_t)SUB ? n - sbase : (size_t)SUB);
  U key[KPL];
#ifdef DRHIP_SORT_STAMPS
  OS_STAMP(2, stamp_clk());
#endif
  load_subtile<DT, XIN, KPL, KPW>(key, src, sbase, valid, lane, wid);
#ifdef DRHIP_SORT_STAMPS
  if (stamp_on) {
    U acc = 0;
#pragma unroll
    for (int r = 0; r < KPL; r++) acc ^= key[r]; // wait for the loads
    st_v[9] = (unsigned long long)acc;
  }
  OS_STAMP(3, stamp_clk());
#endif
  uint32_t rank2[(KPL + 1) / 2];
  rank_subtile<AR, U, KPL, KPW>(key, rank2, valid, (unsigned)SUB, shift, sm.wcnt[wid], lane, wid);
#ifdef DRHIP_SORT_STAMPS
  OS_STAMP(4, stamp_clk());
#endif
  __syncthreads();
  digit_offsets(sm, tid);
#ifdef DRHIP_SORT_STAMPS
  OS_STAMP(5, stamp_clk());
#endif
  // ---- thread d: publish this tile's count of digit d, issue the first
  //      look-back loads, reorder the keys in LDS while they are in flight,
  //      then finish the look-back
  const int d = tid;
  const uint32_t cnt = sm.sub[d];
  using SW = std::conditional_t<W32, uint32_t, uint64_t>;
  SW *status = (SW *)status_v;
  SW *row = status + (size_t)tile * kRadix + d;
  // word = flag | value; flag bits: W32 31:30, else (epoch << 2 | flag) << 32
  const SW f_agg = W32 ? (SW)kOsAgg << 30 : (SW)((epoch << 2) | kOsAgg) << 32;
  const SW f_incl = W32 ? (SW)kOsIncl << 30 : (SW)((epoch << 2) | kOsIncl) << 32;
  if (!XIN) __hip_atomic_store(row, (tile ? f_agg : f_incl) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (W32 && status_next) status_next[(size_t)tile * kRadix + d] = 0u;
  // the next digit position's counts: DRHIP_SORT_CNT_WO = 1 counts the
  // reordered keys during the write-out (LDS atomics under the scattered
  // stores), 0 one chunk of the register keys per look-back round trip
  constexpr bool kCntWO = DRHIP_SORT_CNT_WO;
  constexpr int kCntCh = 16, kCntN = kCntWO ? 0 : (KPL + kCntCh - 1) / kCntCh;
  int cnt_chunk = 0;
  auto count_next = [&]() {
    if constexpr (NXT) {
#pragma unroll
      for (int c = 0; c < kCntN; c++)
        if (c == cnt_chunk) {
#pragma unroll
          for (int r = c * kCntCh; r < (c + 1) * kCntCh && r < KPL; r++) {
            const unsigned li = wid * KPW + r * kWave + lane;
            if (li < valid) atomicAdd(&s_nxt[wid][(unsigned)(key[r] >> (shift + 8)) & 0xFF], 1u);
          }
        }
      cnt_chunk++;
    }
  };
  long t = (long)tile - 1;
  SW w[kOsLook];
  auto issue = [&]() {
#pragma unroll
    for (int k = 0; k < kOsLook; k++)
      w[k] = t - k >= 0 ? __hip_atomic_load(status + (size_t)(t - k) * kRadix + d, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : f_incl;
  };
  if (!XIN && tile) issue();
  reorder_keys<U, SUB, KPL, KPW>(sm, key, rank2, valid, shift, lane, wid);
  uint32_t prefix = 0;
  if (!XIN && tile) {
    unsigned spins = 0;
    while (true) {
      int k = 0;
      bool done = false;
#pragma unroll
      for (; k < kOsLook; k++) {
        unsigned flag;
        uint32_t val;
        if constexpr (W32) {
          flag = (uint32_t)w[k] >> 30;
          val = (uint32_t)w[k] & 0x3FFFFFFFu;
        } else {
          const uint32_t hi = (uint32_t)(w[k] >> 32);
          flag = (hi >> 2) == epoch ? (hi & 3u) : 0u;
          val = (uint32_t)w[k];
        }
        if (flag == 0) break; // not yet published
        prefix += val;
        if (flag == kOsIncl) {
          done = true;
          break;
        }
      }
      if (done) break;
#ifdef DRHIP_SORT_STAMPS
      trips++;
#endif
      t -= k;
      if (k < kOsLook) {
#ifdef DRHIP_SORT_STAMPS
        waits++;
#endif
        if (++spins > kOsSpinLimit) {
          __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      issue();
      if (NXT && cnt_chunk < kCntN) count_next();
    }
    __hip_atomic_store(row, f_incl | (SW)(prefix + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (NXT)
    while (cnt_chunk < kCntN) count_next();
#ifdef DRHIP_SORT_STAMPS
  OS_STAMP(6, stamp_clk());
#endif
  // key p of the reordered tile goes to s_run[d] + p
  s_run[d] = (XIN ? pre[(size_t)tile * kRadix + d] : dstart[d] + prefix) - sm.start[d];
  __syncthreads();
  if constexpr (NXT && !kCntWO) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < kSortWaves; w++) c += s_nxt[w][d];
    if (c) atomicAdd(nxt_hist + (size_t)(tile % kOsHistParts) * kRadix + d, c);
  }
#ifdef DRHIP_SORT_STAMPS
  OS_STAMP(7, stamp_clk());
#endif
#pragma unroll
  for (int r = 0; r < KPL; r++) {
    const unsigned p = r * kSortThreads + tid;
    if (p < valid) {
      const U k = sm.keys[p];
      const unsigned d = (unsigned)(k >> shift) & 0xFF;
#if defined(DRHIP_SORT_WRITE_MODE) && DRHIP_SORT_WRITE_MODE == 0 // measurement: no global stores
      if (k == (U)0x9E3779B9u && n == 3) dst[p] = k;
#elif defined(DRHIP_SORT_WRITE_MODE) && DRHIP_SORT_WRITE_MODE == 2 // measurement: coalesced stores
      dst[sbase + p] = XOUT ? KeyBits<DT>::out(k) : k + (U)s_run[d];
#else
      dst[s_run[d] + p] = XOUT ? KeyBits<DT>::out(k) : k;
#endif
      if (NXT && kCntWO) atomicAdd(&s_nxt[wid][(unsigned)(k >> (shift + 8)) & 0xFF], 1u);
    }
  }
  if constexpr (NXT && kCntWO) {
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < kSortWaves; w++) c += s_nxt[w][d];
    if (c) atomicAdd(nxt_hist + (size_t)(tile % kOsHistParts) * kRadix + d, c);
  }
#ifdef DRHIP_SORT_STAMPS
  if (stamp_on && tile < kStampTiles) {
    st_v[8] = stamp_rt();
    st_v[9] = trips | ((unsigned long long)waits << 32) | ((unsigned long long)(st_v[9] & 1) << 63);
    for (int k = 0; k < kStampSlots; k++) g_sort_stamps[(size_t)tile * kStampSlots + k] = st_v[k];
  }
#endif
}

// XCD-grouped persistent form of radix_onesweep, the default for 4-byte
// keys (DRHIP_SORT_OS_PT=0 selects the one-shot kernel).  Grid = resident
// blocks; the blocks of one XCD (HW_REG_XCC_ID) take their tiles from that
// XCD's counter in groups of kOsGroup consecutive tiles (XCD x owns groups
// x, x + 8, ...), so the tiles writing either side of a digit run's
// boundary line mostly run on the same XCD at the same time and their
// partial lines merge in that XCD's L2 before write-back.  2^28 u32
// (tools/sort_group.sh): one-shot 2.93 ms; groups of 8 / 16 / 32 / 64
// tiles 2.72 / 2.74 / 2.79 / 2.68 ms; 128 / 256 (more than an XCD's 64
// resident blocks) 8.2 / 10.9 ms.  Each XCD walks its own tiles in
// increasing order and every XCD has resident blocks, so the lowest
// unfinished tile is always claimed and its look-back only reads lower
// tiles.  A persistent form that also loaded the next tile during the
// write-out ran slower (pass 0 0.60 -> 0.67 ms): the passes are bound by
// the memory system under the scattered stores, not by load latency.
constexpr int kOsGroup = 64;
// DRHIP_SORT_EARLY_PUB=1 (measurement knob): passes 1-3 publish a tile's
// digit counts (AGG) from the per-wave counts right after ranking, before
// the digit scan.  Round 5, 2^28 u32, interleaved with the default on one
// box (profiles/r05_sort_early_pub_ab.txt): see DESIGN 4.0.
#ifndef DRHIP_SORT_EARLY_PUB
#define DRHIP_SORT_EARLY_PUB 0
#endif
constexpr bool kOsEarlyPub = DRHIP_SORT_EARLY_PUB;
#ifndef DRHIP_SORT_P0_ONESHOT
#define DRHIP_SORT_P0_ONESHOT 0
#endif
constexpr bool kOsP0OneShot = DRHIP_SORT_P0_ONESHOT;
template <int DT, bool XIN, bool XOUT, bool BIG, bool AR, bool W32, int NT = kSortThreads>
__global__ __launch_bounds__(NT, (OsCfg<typename KeyBits<DT>::U, BIG, NT>::MINW)) void radix_onesweep_pt(
    const typename KeyBits<DT>::U *src, typename KeyBits<DT>::U *dst, size_t n, int shift, const uint32_t *dstart,
    const uint32_t *pre, void *status_v, uint32_t *status_next, uint32_t *nxt_hist, unsigned *xcd_counter,
    unsigned tiles, unsigned group, unsigned nxcd, unsigned xmask, uint32_t *lstatus, uint32_t *lstatus_next,
    unsigned local, unsigned *err) {
  using U = typename KeyBits<DT>::U;
  using Cfg = OsCfg<U, BIG, NT>;
  constexpr int NW = Cfg::NW;
  constexpr int KPL = Cfg::KPL;
  constexpr int SUB = Cfg::SUB;
  constexpr int KPW = SUB / NW;
  constexpr bool NXT = !XOUT && !(XIN && kH0Cnt1) && !kH0All;
  using SW = std::conditional_t<W32, uint32_t, uint64_t>;
  static_assert(W32, "the grouped onesweep uses the 4-byte status words");
  constexpr SW f_agg = (SW)kOsAgg << 30, f_incl = (SW)kOsIncl << 30;

  __shared__ RankSmem<U, SUB, NW> sm;
  __shared__ uint32_t s_run[kRadix];
  __shared__ uint32_t s_nxt[NXT ? NW : 1][kRadix];
  __shared__ unsigned s_tile;

  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave, d = tid;
  SW *status = (SW *)status_v;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // dense index of this XCD among the ids the device's probe saw (os_xcd):
  // every one of the nxcd counters is claimed by blocks of a present XCD
  xcc = nxcd > 1 ? (unsigned)__builtin_popcount(xmask & ((1u << (xcc & 0xF)) - 1u)) % nxcd : 0u;
  if constexpr (NXT)
    for (int i = tid; i < NW * kRadix; i += NT) (&s_nxt[0][0])[i] = 0;
  // pass 0 (XIN) has no look-back, so it needs no claim order: with
  // kOsP0OneShot it is a one-shot grid, block b taking tile b through the
  // same XCD grouping under round-robin dispatch (b -> XCD b % 8; a wrong
  // guess only loses the grouping, never correctness)
  constexpr bool ONESHOT = XIN && kOsP0OneShot;
  // the few-digit ranking (kSortFewK) only in a pass whose histogram has a
  // digit holding at least a quarter of the keys (dstart: this position's
  // digit starts over the whole input): no per-tile probe otherwise
  bool few_ok = false;
  if constexpr (kSortFewK > 0) {
    __shared__ uint32_t s_maxc;
    if (tid == 0) s_maxc = 0;
    __syncthreads();
    if (d < kRadix) atomicMax(&s_maxc, (d < kRadix - 1 ? dstart[d + 1] : (uint32_t)n) - dstart[d]);
    __syncthreads();
    few_ok = (size_t)s_maxc * 4 >= n;
  }
  bool done_once = false;
  while (true) {
    if (tid == 0) {
      if constexpr (ONESHOT) {
        const unsigned b = blockIdx.x, full = tiles / (8 * group) * (8 * group);
        const unsigned j = b / 8;
        s_tile = done_once ? ~0u : b < full ? ((j / group) * 8 + b % 8) * group + j % group : b;
      } else {
        const unsigned c = atomicAdd(xcd_counter + xcc, 1u);
        s_tile = ((c / group) * nxcd + xcc) * group + c % group;
      }
    }
    done_once = true;
    for (int i = tid; i < NW * kDigits1; i += NT) (&sm.wcnt[0][0])[i] = 0;
    __syncthreads();
    const unsigned tile = s_tile;
    if (tile >= tiles) break; // block-uniform; later claims are larger
    const size_t sbase = (size_t)tile * SUB;
    const unsigned valid = (unsigned)(n - sbase < (size_t)SUB ? n - sbase : (size_t)SUB);
    U key[KPL];
    load_subtile<DT, XIN, KPL, KPW>(key, src, sbase, valid, lane, wid);
    uint32_t rank2[(KPL + 1) / 2];
    rank_subtile<AR, U, KPL, KPW>(key, rank2, valid, (unsigned)SUB, shift, sm.wcnt[wid], lane, wid, few_ok);
    __syncthreads();
    if constexpr (kOsEarlyPub) {
      // the tile's digit counts (AGG) straight from the per-wave counts,
      // before the digit scan's two barriers (measurement knob, see kOsEarlyPub)
      if (!XIN && tile && d < kRadix) {
        uint32_t c = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) c += sm.wcnt[ww][d];
        __hip_atomic_store(status + (size_t)tile * kRadix + d, f_agg | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (local)
          __hip_atomic_store(lstatus + (size_t)tile * kRadix + d, (uint32_t)(f_agg | c), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    digit_offsets(sm, tid);
    // thread d < 256 owns digit d's publication, look-back and cursor
    const bool dig = d < kRadix;
    const uint32_t cnt = dig ? sm.sub[d] : 0u;
    SW *row = status + (size_t)tile * kRadix + d;
    uint32_t *lrow = lstatus + (size_t)tile * kRadix + d;
    // Two copies of each status word: `status` by an agent-scope store
    // (written through to memory, dropped from this XCD's L2: what a reader
    // on ANOTHER XCD needs), `lstatus` by a plain store, which stays in this
    // XCD's L2 -- every tile of the same group runs on this XCD, and its
    // agent-scope (L1-bypassing) loads of that copy are served by this L2
    // instead of the memory side.  A stale read only ever returns an older
    // state of the word (0 -> AGG -> INCL, each payload final), which the
    // look-back handles (it re-polls or walks further back); the copies
    // of the next pass are zeroed here, ordered by the kernel boundary.
    const long gfirst = (long)(tile / group) * group; // first tile of this XCD group
    auto publish = [&](SW word) {
      __hip_atomic_store(row, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (local) __hip_atomic_store(lrow, (uint32_t)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if (!XIN && dig && !(kOsEarlyPub && tile)) publish((tile ? f_agg : f_incl) | cnt);
    if (status_next && dig) status_next[(size_t)tile * kRadix + d] = 0u;
    if (lstatus_next && dig) lstatus_next[(size_t)tile * kRadix + d] = 0u;
    long t = (long)tile - 1;
    SW w[kOsLook];
    auto issue = [&]() {
#pragma unroll
      for (int k = 0; k < kOsLook; k++) {
        const long q = t - k;
        const SW *src = (local && q >= gfirst) ? (const SW *)lstatus : status;
        w[k] = q >= 0 ? __hip_atomic_load(src + (size_t)q * kRadix + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : f_incl;
      }
    };
    if (!XIN && tile && dig) issue();
    reorder_keys<U, SUB, KPL, KPW, NW>(sm, key, rank2, valid, shift, lane, wid);
    uint32_t prefix = 0;
    if (!XIN && tile && dig) {
      unsigned spins = 0;
      while (true) {
        int k = 0;
        bool done = false;
#pragma unroll
        for (; k < kOsLook; k++) {
          const unsigned flag = (uint32_t)w[k] >> 30;
          if (flag == 0) break; // not yet published
          prefix += (uint32_t)w[k] & 0x3FFFFFFFu;
          if (flag == kOsIncl) {
            done = true;
            break;
          }
        }
        if (done) break;
        t -= k;
        if (k < kOsLook) {
          if (++spins > kOsSpinLimit) {
            __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        issue();
      }
      publish(f_incl | (SW)(prefix + cnt));
    }
    if (dig) s_run[d] = (XIN ? pre[(size_t)tile * kRadix + d] : dstart[d] + prefix) - sm.start[d];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned p = r * NT + tid;
      if (p < valid) {
        const U k = sm.keys[p];
#if defined(DRHIP_SORT_NT_STORE) && DRHIP_SORT_NT_STORE // measurement: nontemporal write-out
        __builtin_nontemporal_store(XOUT ? KeyBits<DT>::out(k) : k, dst + s_run[(unsigned)(k >> shift) & 0xFF] + p);
#else
        dst[s_run[(unsigned)(k >> shift) & 0xFF] + p] = XOUT ? KeyBits<DT>::out(k) : k;
#endif
        if (NXT) {
          const unsigned nd = (unsigned)(k >> (shift + 8)) & 0xFF;
          if constexpr (kSortUniNxt) {
            // the wave's active lanes all on one next digit: one add
            const unsigned ndw = __builtin_amdgcn_readfirstlane(nd);
            if (__all(nd == ndw)) {
              if (__builtin_amdgcn_readfirstlane(lane) == (unsigned)lane)
                atomicAdd(&s_nxt[wid][ndw], (uint32_t)__builtin_popcountll(__ballot(1)));
            } else {
              atomicAdd(&s_nxt[wid][nd], 1u);
            }
          } else {
            atomicAdd(&s_nxt[wid][nd], 1u);
          }
        }
      }
    }
    __syncthreads();
    if constexpr (NXT) {
      // column d is read and cleared by thread d only
      if (dig) {
        uint32_t c = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
          c += s_nxt[ww][d];
          s_nxt[ww][d] = 0;
        }
        if (c) atomicAdd(nxt_hist + (size_t)(tile % kOsHistParts) * kRadix + d, c);
      }
    }
  }
}

// ------------------------------------------------ sample-sort helpers
// regular samples of a sorted run: samples[j] = sorted[j * stride],
// j < ceil(n / stride) (the input of drhip_split_windows, split.hip)
template <typename K>
__global__ void sample_kernel(const K *sorted, size_t n, size_t stride, size_t count, K *samples) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < count) samples[i] = sorted[i * stride];
}

// counts[b] = #keys in [splitter[b-1], splitter[b]) (b = 0..nsplit), keys
// compared in the radix order (order-preserving bits: std::less for every
// non-NaN key, -0.0 before +0.0), the order drhip_sort produces.
template <int DT>
__global__ void bucket_count_kernel(const typename KeyBits<DT>::U *sorted, size_t n,
                                    const typename KeyBits<DT>::U *spl, int nsplit, uint64_t *counts) {
  const int b = threadIdx.x;
  if (b > nsplit) return;
  // lower_bound of splitter b-1 and splitter b
  auto lower = [&](int s) -> size_t {
    if (s < 0) return 0;
    if (s >= nsplit) return n;
    const auto v = KeyBits<DT>::in(spl[s]);
    size_t lo = 0, hi = n;
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      if (KeyBits<DT>::in(sorted[mid]) < v) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  counts[b] = lower(b) - lower(b - 1);
}

// ------------------------------------------------------ merge of sorted runs
// The distributed sort's destination step: after the all-to-all every rank
// holds P sorted runs (one from each source), which pairwise merge-path
// rounds (ceil(log2 P) passes of 8 B/key for 4-byte keys) put in order
// instead of a second full radix sort (48 B/key).  Keys only, so ties need
// no stability; runs of pair p are A (earlier) and B, A first on ties.
constexpr int kMergeThreads = 256;
constexpr int kMergeIPT = 8; // outputs per thread
constexpr int kMergeTile = kMergeThreads * kMergeIPT;
constexpr int kMaxMergePairs = 64;
struct MergePairs {
  unsigned long long a0[kMaxMergePairs], alen[kMaxMergePairs], blen[kMaxMergePairs];
  unsigned tile0[kMaxMergePairs + 1]; // first global tile of pair p; tile0[npairs] = total tiles
  int npairs;
};

template <int DT> __device__ __forceinline__ bool merge_le(typename KeyBits<DT>::U x, typename KeyBits<DT>::U y) {
  return KeyBits<DT>::in(x) <= KeyBits<DT>::in(y);
}

// merge-path co-rank: how many of the first d merged outputs come from A
template <int DT, typename P>
__device__ __forceinline__ size_t merge_corank(P A, size_t m, P B, size_t k, size_t d) {
  size_t lo = d > k ? d - k : 0, hi = d < m ? d : m;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (merge_le<DT>(A[mid], B[d - mid - 1])) lo = mid + 1; // A[mid] goes first
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int merge_pair_of(const MergePairs &mp, unsigned g) {
  int p = 0;
  while (p + 1 < mp.npairs && mp.tile0[p + 1] <= g) p++;
  return p;
}

// split[g + p] = co-rank at pair p's tile boundary g - tile0[p] (inclusive of
// the pair's end boundary)
template <int DT>
__global__ void merge_partition(const typename KeyBits<DT>::U *src, MergePairs mp, unsigned long long *split) {
  const unsigned nb = mp.tile0[mp.npairs] + (unsigned)mp.npairs;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb) return;
  // boundary t belongs to the pair p with tile0[p] + p <= t <= tile0[p+1] + p
  int p = 0;
  while (p + 1 < mp.npairs && mp.tile0[p + 1] + (unsigned)(p + 1) <= t) p++;
  const size_t m = mp.alen[p], k = mp.blen[p];
  const size_t d0 = (size_t)(t - mp.tile0[p] - (unsigned)p) * kMergeTile;
  const size_t d = d0 < m + k ? d0 : m + k;
  const auto *A = src + mp.a0[p];
  split[t] = merge_corank<DT>(A, m, A + m, k, d);
}

template <int DT>
__global__ __launch_bounds__(kMergeThreads) void merge_tiles(const typename KeyBits<DT>::U *src,
                                                            typename KeyBits<DT>::U *dst, MergePairs mp,
                                                            const unsigned long long *split) {
  using U = typename KeyBits<DT>::U;
  __shared__ U s_a[kMergeTile], s_b[kMergeTile];
  const unsigned g = blockIdx.x;
  const int p = merge_pair_of(mp, g);
  const size_t m = mp.alen[p], k = mp.blen[p];
  const size_t d0 = (size_t)(g - mp.tile0[p]) * kMergeTile;
  const size_t d1 = d0 + kMergeTile < m + k ? d0 + kMergeTile : m + k;
  const size_t i0 = split[g + p], i1 = split[g + p + 1];
  const size_t j0 = d0 - i0, j1 = d1 - i1;
  const unsigned na = (unsigned)(i1 - i0), nbk = (unsigned)(j1 - j0), tot = (unsigned)(d1 - d0);
  const U *A = src + mp.a0[p], *B = A + m;
  for (unsigned x = threadIdx.x; x < na; x += kMergeThreads) s_a[x] = A[i0 + x];
  for (unsigned x = threadIdx.x; x < nbk; x += kMergeThreads) s_b[x] = B[j0 + x];
  __syncthreads();
  const unsigned od = threadIdx.x * kMergeIPT;
  if (od >= tot) return;
  // co-rank of this thread's first output inside the tile
  unsigned lo = od > nbk ? od - nbk : 0, hi = od < na ? od : na;
  while (lo < hi) {
    const unsigned mid = (lo + hi) / 2;
    if (merge_le<DT>(s_a[mid], s_b[od - mid - 1])) lo = mid + 1;
    else hi = mid;
  }
  unsigned ia = lo, ib = od - lo;
  U out[kMergeIPT];
#pragma unroll
  for (int q = 0; q < kMergeIPT; q++) {
    const bool take_a = ib >= nbk || (ia < na && merge_le<DT>(s_a[ia], s_b[ib]));
    out[q] = take_a ? s_a[ia < na ? ia : 0] : s_b[ib < nbk ? ib : 0];
    ia += take_a;
    ib += !take_a;
  }
  U *o = dst + mp.a0[p] + d0 + od;
  const unsigned cnt = tot - od < (unsigned)kMergeIPT ? tot - od : (unsigned)kMergeIPT;
  if (cnt == (unsigned)kMergeIPT && ((uintptr_t)o % 16) == 0) {
    constexpr int V = 16 / sizeof(U);
#pragma unroll
    for (int q = 0; q < kMergeIPT; q += V) {
      Vec16<U> v;
#pragma unroll
      for (int j = 0; j < V; j++) v.v[j] = out[q + j];
      *reinterpret_cast<Vec16<U> *>(o + q) = v;
    }
  } else {
    for (unsigned q = 0; q < cnt; q++) o[q] = out[q];
  }
}

template <int DT> static int launch_sort(Segment *s, int seg, void *keys, size_t n, void *tmp, size_t tmp_bytes);

} // namespace drhip

using namespace drhip;

namespace {

template <typename U> bool sort_big(size_t n) { return n * sizeof(U) >= kSortBigBytes; }
template <typename U> size_t sort_nblocks(size_t n) {
  const size_t ch = sort_big<U>(n) ? SortCfg<U, true>::CH : SortCfg<U, false>::CH;
  return (n + ch - 1) / ch;
}

// Path choice, read at every call (so tests can switch it): onesweep with
// the big sub-tile from kSortBigBytes of keys (2^28 u32: 3.92-4.04 ms vs
// 4.16 ms classic), the classic per-pass-histogram path below (2^24 u32:
// 0.317 ms classic vs 0.397 ms onesweep).  DRHIP_SORT_ALGO=classic|onesweep
// forces one; DRHIP_SORT_OS_SHAPE=small picks the 4 K-key onesweep tile
// (5.5-5.7 ms at 2^28: more tiles, more look-back).  tools/sort_os_run.sh.
template <typename U> bool sort_onesweep(size_t n) {
  const char *e = getenv("DRHIP_SORT_ALGO");
  if (e && !strcmp(e, "classic")) return false;
  if (e && !strcmp(e, "onesweep")) return true;
  return sort_big<U>(n);
}
bool sort_os_big() {
  const char *e = getenv("DRHIP_SORT_OS_SHAPE");
  return !(e && !strcmp(e, "small"));
}
template <typename U> size_t os_sub(bool big) { return big ? OsCfg<U, true>::SUB : OsCfg<U, false>::SUB; }
// onesweep control block: tile counters, digit starts [P][256], the
// next-digit partial histograms [P][kOsHistParts][256]
template <typename U> constexpr size_t os_ctrl_bytes() {
  return (256 + sizeof(U) * kRadix * 4 + sizeof(U) * kOsHistParts * kRadix * 4 + 255) & ~size_t(255);
}
// per-sort arrays, sized for the smaller sub-tile so either shape fits:
// status words (one array of 8-byte words or two of 4-byte words), the
// pass-0 tile bases [tiles][256] and the chunk bases [chunks][256]
template <typename U> size_t os_tiles_max(size_t n) { return (n + os_sub<U>(false) - 1) / os_sub<U>(false); }
template <typename U> size_t os_chunks_max(size_t n) { return os_tiles_max<U>(n) / kOsChunk + 1; }
template <typename U> size_t os_status_bytes(size_t n) {
  // + two 4-byte arrays of same-XCD status words (radix_onesweep_pt)
  return os_tiles_max<U>(n) * kRadix * (8 + 4 + 8) + os_chunks_max<U>(n) * kRadix * 4;
}
// XCD-grouped persistent onesweep (radix_onesweep_pt) unless DRHIP_SORT_OS_PT=0
bool os_persistent() {
  const char *e = getenv("DRHIP_SORT_OS_PT");
  return !(e && !strcmp(e, "0"));
}
// XCDs sharing the device's blocks, found from the hardware: a probe grid
// of 4 blocks per CU records every HW_REG_XCC_ID its blocks ran on (8 ids on
// an MI355X in SPX mode; 4 / 2 / 1 in the DPX / QPX / CPX partitions, whose
// ids need not start at 0).  The kernel maps an id to its dense index
// among the probed ids, so every counter it claims from belongs to an XCD
// that hosts blocks.  More than 8 ids (the control block holds 8 counters
// per pass) or a failed probe -> 1 (plain start-order claims).
// DRHIP_SORT_OS_NXCD=k (tests) folds the dense indices onto min(k, ids)
// counters.
__global__ void xcc_probe_kernel(unsigned *mask) {
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    atomicOr(mask, 1u << (xcc & 0xF));
  }
}
struct XcdInfo {
  unsigned nxcd, mask;
  bool one_xcd_per_counter; // every counter's groups run on ONE XCD (the same-XCD status copy needs it)
};
XcdInfo os_xcd(Segment *s) {
  static unsigned probed[256]; // (mask + 1) per device, 0 = not probed
  const int dev = s->device & 255;
  if (!probed[dev]) {
    unsigned *v = nullptr, hv = 0;
    if (hipMalloc(&v, sizeof(unsigned)) == hipSuccess) {
      if (hipMemsetAsync(v, 0, sizeof(unsigned), s->stream) == hipSuccess) {
        hipLaunchKernelGGL(xcc_probe_kernel, dim3((unsigned)s->num_cus * 4), dim3(64), 0, s->stream, v);
        if (hipMemcpyAsync(&hv, v, sizeof(unsigned), hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess)
          hv = 0;
      }
      (void)hipFree(v);
    }
    (void)hipGetLastError();
    probed[dev] = hv + 1;
  }
  const unsigned mask = probed[dev] - 1;
  const int ids = __builtin_popcount(mask);
  if (ids < 2 || ids > 8) return {1u, 0u, false};
  unsigned k = (unsigned)ids;
  if (const char *e = getenv("DRHIP_SORT_OS_NXCD")) {
    const int f = atoi(e);
    if (f >= 1 && f < ids) k = (unsigned)f;
  }
  // folded counters are claimed from several XCDs: a plain-store status copy
  // in one XCD's L2 is invisible to the others, so only the agent-scope
  // copy may be read then
  return {k, mask, k == (unsigned)ids};
}
// same-XCD look-back through the L2-resident status copy unless
// DRHIP_SORT_OS_LOCAL=0 (and only where groups are pinned to XCDs)
unsigned os_local() {
  const char *e = getenv("DRHIP_SORT_OS_LOCAL");
  return (e && e[0] == '0') ? 0u : 1u;
}
// tiles per XCD group (DRHIP_SORT_OS_GROUP): kOsGroup at 256 threads, one
// tile per resident block of an XCD (32) at 512 -- a group larger than the
// blocks an XCD holds serialises its claims (DESIGN.md sort notes)
unsigned os_group(int nt) {
  const char *e = getenv("DRHIP_SORT_OS_GROUP");
  const int g = e ? atoi(e) : 0;
  return g > 0 ? (unsigned)g : (unsigned)(nt == 512 ? kOsGroup / 2 : kOsGroup);
}
// resident blocks of a persistent kernel on this device (cached per kernel)
template <auto K, int NT = kSortThreads> unsigned os_pt_grid(Segment *s, size_t tiles) {
  static int per_cu = 0;
  if (!per_cu) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, K, NT, 0) != hipSuccess || b < 1) b = 1;
    per_cu = b;
  }
  (void)tiles; // every XCD needs resident blocks: the full resident grid
  return (unsigned)((size_t)s->num_cus * per_cu);
}
// threads per block of the XCD-grouped onesweep: 256 (16 K-key tiles, two
// blocks per CU) unless DRHIP_SORT_OS_NT=512 (32 K-key tiles, one per CU).
// Round 4, 2^28 u32, three interleaved pairs on one box
// (profiles/r04_sort_nt_ab.txt): 512 -> 2.80-2.81 ms, 256 -> 2.72-2.75 ms.
// Per pass (rocprof): pass 0 0.624 vs 0.558 ms (one block per CU leaves a
// CU idle between its block's memory phases), middle passes 0.683 vs 0.681,
// last 0.623 vs 0.625 (half the tiles and look-back round trips per key
// buy back exactly what the lost overlap costs), tile histogram 0.179 vs
// 0.201.  So the look-back is not what bounds passes 1-3.
int os_nt() {
  const char *e = getenv("DRHIP_SORT_OS_NT");
  return (e && !strcmp(e, "512")) ? 512 : 256;
}
// DRHIP_SORT_STATUS=w64 keeps the 8-byte words at any size (tests, sweeps)
bool os_force_w64() {
  const char *e = getenv("DRHIP_SORT_STATUS");
  return e && !strcmp(e, "w64");
}

template <typename U> size_t sort_ws_bytes(size_t n) {
  const size_t nb = sort_nblocks<U>(n);
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  const size_t hist_b = (nb * kRadix * 4 + 255) & ~size_t(255);
  const size_t os_b = os_ctrl_bytes<U>() + os_status_bytes<U>(n);
  return keys_b + (2 * hist_b > os_b ? 2 * hist_b : os_b);
}

template <typename F> int dispatch_sort_dtype(int dtype, F &&f) {
  switch (dtype) {
  case DRHIP_U32: return f(std::integral_constant<int, DRHIP_U32>{});
  case DRHIP_I32: return f(std::integral_constant<int, DRHIP_I32>{});
  case DRHIP_F32: return f(std::integral_constant<int, DRHIP_F32>{});
  case DRHIP_U64: return f(std::integral_constant<int, DRHIP_U64>{});
  case DRHIP_I64: return f(std::integral_constant<int, DRHIP_I64>{});
  case DRHIP_F64: return f(std::integral_constant<int, DRHIP_F64>{});
  default: return set_error(DRHIP_ERR_BAD_ARG, "sort: unsupported dtype");
  }
}

// The atomic ranking (rank_keys_atomic) relies on ds_add_rtn_u32 returning
// the old values of same-address lanes in lane order.  Checked once per
// device before the first sort, at the occupancy of the sort passes (2
// blocks per CU: 64 KiB of padding LDS per block, every CU filled) and at
// the full 8 blocks per CU: 32 rounds of counter adds over 1, 4, 16, 64 and
// 256 distinct counters per wave; any lane pair out of order selects the
// ballot ranking for that device.
__global__ __launch_bounds__(256) void lds_rank_order_probe(unsigned *viol) {
  extern __shared__ uint32_t pad[]; // occupancy only
  if (threadIdx.x == 0 && viol == nullptr) pad[0] = 0;
  __shared__ uint32_t cnt[kSortWaves][kDigits1];
  __shared__ uint32_t got[kSortWaves][kWave], dig[kSortWaves][kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  for (int i = tid; i < kSortWaves * kDigits1; i += 256) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const unsigned range = 1u << (2 * (blockIdx.x % 5)); // 1, 4, 16, 64, 256 counters
  unsigned bad = 0;
  for (int r = 0; r < 32; r++) {
    uint32_t h = (uint32_t)(blockIdx.x * 7919u + r * 104729u + tid * 2654435761u);
    h ^= h >> 15;
    h *= 0x2c1b3c6dU;
    h ^= h >> 12;
    const unsigned d = h % range;
    const uint32_t old = atomicAdd(&cnt[w][d], 1u);
    got[w][lane] = old;
    dig[w][lane] = d;
    __syncthreads();
    for (int j = 0; j < lane; j++)
      if (dig[w][j] == d && !(got[w][j] < old)) bad++;
    __syncthreads();
  }
  if (bad) atomicAdd(viol, bad);
}

bool sort_rank_atomic(Segment *s) {
  const char *e = getenv("DRHIP_SORT_RANK");
  if (e && !strcmp(e, "ballot")) return false;
  if (e && !strcmp(e, "atomic")) return true;
  static int known[256];        // 0 unknown, 1 ordered, 2 not ordered
  const int dev = s->device & 255;
  if (!known[dev]) {
    unsigned *v = nullptr, hv = 1;
    if (hipMalloc(&v, sizeof(unsigned)) == hipSuccess) {
      if (hipMemsetAsync(v, 0, sizeof(unsigned), s->stream) == hipSuccess) {
        const unsigned cus = (unsigned)(s->num_cus > 0 ? s->num_cus : 256);
        // a probe launch that fails (e.g. an arch that caps a workgroup's
        // LDS below the 64 KiB of padding) leaves the ordering unverified at
        // the passes' occupancy: ballot ranking then
        hipLaunchKernelGGL(lds_rank_order_probe, dim3(2 * cus), dim3(256), 64 * 1024, s->stream, v);
        const bool l1 = hipGetLastError() == hipSuccess;
        hipLaunchKernelGGL(lds_rank_order_probe, dim3(8 * cus), dim3(256), 0, s->stream, v);
        const bool l2 = hipGetLastError() == hipSuccess;
        if (hipMemcpyAsync(&hv, v, sizeof(unsigned), hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess || !l1 || !l2)
          hv = 1;
      }
      (void)hipFree(v);
    }
    (void)hipGetLastError();
    known[dev] = hv == 0 ? 1 : 2;
  }
  return known[dev] == 1;
}

} // namespace

template <int DT, bool BIG, bool AR> static int launch_sort_cfg(Segment *s, int seg, void *keys, size_t n, void *tmp);
template <int DT, bool BIG, bool AR, int NT = kSortThreads>
static int launch_onesweep(Segment *s, int seg, void *keys, size_t n, void *tmp);

template <int DT> int drhip::launch_sort(Segment *s, int seg, void *keys, size_t n, void *tmp, size_t tmp_bytes) {
  using U = typename KeyBits<DT>::U;
  if (n <= 1) return DRHIP_OK;
  if (n >= (size_t(1) << 32)) return set_error(DRHIP_ERR_BAD_ARG, "sort: segment must hold < 2^32 keys");
  if (((uintptr_t)keys % sizeof(U)) || ((uintptr_t)tmp & 255))
    return set_error(DRHIP_ERR_BAD_ARG, "sort: keys must be key-aligned and tmp 256-byte aligned");
  if (tmp_bytes < sort_ws_bytes<U>(n)) return set_error(DRHIP_ERR_BAD_ARG, "sort: workspace too small");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const bool ar = sort_rank_atomic(s);
  if (sort_onesweep<U>(n)) {
    // 512-thread tiles: the grouped (persistent) form, 4-byte keys below 2^30
    if (sort_os_big() && sizeof(U) == 4 && os_persistent() && os_nt() == 512 && n < (size_t(1) << 30) &&
        !os_force_w64())
      return ar ? launch_onesweep<DT, true, true, 512>(s, seg, keys, n, tmp)
                : launch_onesweep<DT, true, false, 512>(s, seg, keys, n, tmp);
    if (sort_os_big())
      return ar ? launch_onesweep<DT, true, true>(s, seg, keys, n, tmp)
                : launch_onesweep<DT, true, false>(s, seg, keys, n, tmp);
    return ar ? launch_onesweep<DT, false, true>(s, seg, keys, n, tmp)
              : launch_onesweep<DT, false, false>(s, seg, keys, n, tmp);
  }
  if (sort_big<U>(n))
    return ar ? launch_sort_cfg<DT, true, true>(s, seg, keys, n, tmp)
              : launch_sort_cfg<DT, true, false>(s, seg, keys, n, tmp);
  return ar ? launch_sort_cfg<DT, false, true>(s, seg, keys, n, tmp)
            : launch_sort_cfg<DT, false, false>(s, seg, keys, n, tmp);
}

template <int DT, bool BIG, bool AR, int NT>
static int launch_onesweep(Segment *s, int seg, void *keys, size_t n, void *tmp) {
  (void)seg;
  using U = typename KeyBits<DT>::U;
  using Cfg = OsCfg<U, BIG, NT>;
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  const size_t tiles = (n + Cfg::SUB - 1) / Cfg::SUB;
  char *ctrl = (char *)tmp + keys_b;
  unsigned *counters = (unsigned *)ctrl;                          // [PASSES]
  uint32_t *dstart = (uint32_t *)(ctrl + 256);                    // [PASSES][256]
  uint32_t *parts = dstart + Cfg::PASSES * kRadix;                // [PASSES][kOsHistParts][256]
  char *status = ctrl + os_ctrl_bytes<U>();                       // [tiles][256] words
  const size_t tmax = os_tiles_max<U>(n);
  uint32_t *tilecnt = (uint32_t *)(status + tmax * kRadix * 8);   // [tiles][256]
  uint32_t *chunksum = tilecnt + tmax * kRadix;                   // [chunks][256]
  const size_t nchunks = (tiles + kOsChunk - 1) / kOsChunk;
  // 4-byte words below 2^30 keys (two alternating arrays, zeroed by the
  // passes themselves), else 8-byte words with the pass epoch (one array)
  const bool w32 = n < (size_t(1) << 30) && !os_force_w64();
  uint32_t *st32[2] = {(uint32_t *)status, (uint32_t *)status + tiles * kRadix};
  uint32_t *lst0 = chunksum + os_chunks_max<U>(n) * kRadix;
  uint32_t *lst[2] = {lst0, lst0 + tiles * kRadix};
  const bool pt = os_persistent() && sizeof(U) == 4; // 8 per-XCD counters per pass in ctrl words 16..47
  const XcdInfo xi = pt ? os_xcd(s) : XcdInfo{1u, 0u, false};
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipMemsetAsync(ctrl, 0, os_ctrl_bytes<U>(), s->stream));
  DRHIP_CHECK_HIP(hipMemsetAsync(chunksum, 0, nchunks * kRadix * 4, s->stream));
  if (!w32) DRHIP_CHECK_HIP(hipMemsetAsync(status, 0, tiles * kRadix * 8, s->stream));
  // pass-0 bases: tile counts of position 0 (+ position 1's histogram),
  // per-digit chunk scan, digit starts, tile scan.  Position 0's digit
  // totals go to parts[0][0] (the other 63 partials stay zero).
  hipLaunchKernelGGL((radix_tile_hist0<DT, BIG, NT>), dim3((unsigned)tiles), dim3(NT), 0, s->stream,
                     (const U *)keys, n, tilecnt, chunksum, parts + (size_t)kOsHistParts * kRadix);
  DRHIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(radix_chunk_bases, dim3(kRadix), dim3(kSortThreads), 0, s->stream, chunksum, (unsigned)nchunks,
                     parts);
  DRHIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(radix_digit_starts_parts, dim3(1), dim3(kRadix), 0, s->stream, (const uint32_t *)parts, dstart);
  DRHIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(radix_tile_bases, dim3((unsigned)nchunks), dim3(kRadix), 0, s->stream, tilecnt,
                     (const uint32_t *)chunksum, (const uint32_t *)dstart, tiles);
  DRHIP_CHECK_LAUNCH();
  U *a = (U *)keys, *b = (U *)tmp;
  // one persistent sort at a time per device (segments sharing a device)
  if (w32 && pt) {
    const int rc = persistent_lane_begin(s);
    if (rc) return rc;
  }
  for (int p = 0; p < Cfg::PASSES; p++) {
    const bool first = p == 0, last = p == Cfg::PASSES - 1;
    if (!first) {
      // digit starts of position p from the previous pass's partials
      hipLaunchKernelGGL(radix_digit_starts_parts, dim3(1), dim3(kRadix), 0, s->stream,
                         (const uint32_t *)(parts + (size_t)p * kOsHistParts * kRadix), dstart + p * kRadix);
      DRHIP_CHECK_LAUNCH();
    }
    uint32_t *nxt = last || kH0All || (first && kH0Cnt1) ? nullptr : parts + (size_t)(p + 1) * kOsHistParts * kRadix;
#define DRHIP_ONESWEEP(XI, XO)                                                                                 \
  do {                                                                                                         \
    if (w32 && pt)                                                                                             \
      hipLaunchKernelGGL((radix_onesweep_pt<DT, XI, XO, BIG, AR, true, NT>),                                   \
                         dim3((XI && kOsP0OneShot) ? (unsigned)tiles                                            \
                                                   : os_pt_grid<radix_onesweep_pt<DT, XI, XO, BIG, AR, true, NT>, NT>(s, tiles)), \
                         dim3(NT), 0, s->stream, a, b, n, 8 * p, dstart + p * kRadix,                          \
                         (const uint32_t *)tilecnt, (void *)st32[p & 1], last ? nullptr : st32[(p + 1) & 1], nxt, \
                         counters + 16 + 8 * p, (unsigned)tiles, os_group(NT), xi.nxcd, xi.mask, lst[p & 1],     \
                         last ? nullptr : lst[(p + 1) & 1], os_local() && xi.one_xcd_per_counter, s->err);             \
    else if constexpr (NT != kSortThreads)                                                                     \
      return set_error(DRHIP_ERR_UNSUPPORTED, "sort: 512-thread tiles need the grouped 4-byte-status form");   \
    else if (w32)                                                                                              \
      hipLaunchKernelGGL((radix_onesweep<DT, XI, XO, BIG, AR, true>), dim3((unsigned)tiles), dim3(kSortThreads), \
                         0, s->stream, a, b, n, 8 * p, dstart + p * kRadix, (const uint32_t *)tilecnt,           \
                         (void *)st32[p & 1], last ? nullptr : st32[(p + 1) & 1], nxt, counters + p,             \
                         (unsigned)(p + 1), s->err);                                                           \
    else                                                                                                       \
      hipLaunchKernelGGL((radix_onesweep<DT, XI, XO, BIG, AR, false>), dim3((unsigned)tiles), dim3(kSortThreads), \
                         0, s->stream, a, b, n, 8 * p, dstart + p * kRadix, (const uint32_t *)tilecnt,           \
                         (void *)status, nullptr, nxt, counters + p, (unsigned)(p + 1), s->err);                \
  } while (0)
    if (first && last) DRHIP_ONESWEEP(true, true);
    else if (first) DRHIP_ONESWEEP(true, false);
    else if (last) DRHIP_ONESWEEP(false, true);
    else DRHIP_ONESWEEP(false, false);
#undef DRHIP_ONESWEEP
    DRHIP_CHECK_LAUNCH();
    std::swap(a, b);
  }
  if (w32 && pt) return persistent_lane_end(s);
  return DRHIP_OK;
}

template <int DT, bool BIG, bool AR> static int launch_sort_cfg(Segment *s, int seg, void *keys, size_t n, void *tmp) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U, BIG>;
  const size_t nb = sort_nblocks<U>(n);
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  const size_t hist_b = (nb * kRadix * 4 + 255) & ~size_t(255);
  U *alt = (U *)tmp;
  uint32_t *hist = (uint32_t *)((char *)tmp + keys_b);
  uint32_t *off = (uint32_t *)((char *)tmp + keys_b + hist_b);
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  U *a = (U *)keys, *b = alt;
  for (int p = 0; p < Cfg::PASSES; p++) {
    const int shift = 8 * p;
    const bool first = p == 0, last = p == Cfg::PASSES - 1;
    const bool al = ((uintptr_t)a & 15) == 0;
    if (first)
      hipLaunchKernelGGL((radix_hist<DT, true, BIG>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, n,
                         shift, hist, (unsigned)nb, al);
    else
      hipLaunchKernelGGL((radix_hist<DT, false, BIG>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, n,
                         shift, hist, (unsigned)nb, al);
    DRHIP_CHECK_LAUNCH();
    int rc = scan_inclusive_u32(s, seg, hist, off, nb * kRadix);
    if (rc) return rc;
#define DRHIP_SCATTER(XI, XO)                                                                          \
  hipLaunchKernelGGL((radix_scatter<DT, XI, XO, BIG, AR>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, \
                     b, n, shift, hist, off, (unsigned)nb)
    if (first && last) DRHIP_SCATTER(true, true);
    else if (first) DRHIP_SCATTER(true, false);
    else if (last) DRHIP_SCATTER(false, true);
    else DRHIP_SCATTER(false, false);
#undef DRHIP_SCATTER
    DRHIP_CHECK_LAUNCH();
    U *t = a;
    a = b;
    b = t;
  }
  // an even number of passes leaves the result in `keys`
  return DRHIP_OK;
}

#ifdef DRHIP_SORT_STAMPS
// diagnostic build only: copy the per-tile stamps (kStampSlots u64 per tile)
extern "C" int drhip_dbg_sort_stamps(void *host, size_t bytes) {
  const size_t b = std::min(bytes, sizeof(g_sort_stamps));
  DRHIP_CHECK_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sort_stamps), b, 0, hipMemcpyDeviceToHost));
  return DRHIP_OK;
}
#endif

extern "C" int drhip_sort_workspace(int seg, int dtype, size_t n, size_t *bytes) {
  if (!bytes) return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort_workspace: null");
  const size_t ks = dtype_size(dtype);
  if (!ks) return set_error(DRHIP_ERR_BAD_ARG, "sort: unsupported dtype");
  *bytes = ks == 4 ? sort_ws_bytes<uint32_t>(n) : sort_ws_bytes<uint64_t>(n);
  return DRHIP_OK;
}

extern "C" int drhip_sort(int seg, int dtype, void *keys, size_t n, void *tmp, size_t tmp_bytes) {
  DRHIP_GET_SEG(s, seg);
  if (n > 1 && (!keys || !tmp)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort: null pointer");
  return dispatch_sort_dtype(dtype, [&](auto dv) -> int {
    constexpr int DT = decltype(dv)::value;
    return launch_sort<DT>(s, seg, keys, n, tmp, tmp_bytes);
  });
}

extern "C" int drhip_sort_sample(int seg, int dtype, const void *sorted, size_t n, size_t stride,
                                 void *samples) {
  DRHIP_GET_SEG(s, seg);
  if (!stride) return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort_sample: zero stride");
  const size_t count = (n + stride - 1) / stride;
  if (!count) return DRHIP_OK;
  if (!sorted || !samples) return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort_sample: bad argument");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using K = decltype(tv);
    hipLaunchKernelGGL((sample_kernel<K>), dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s->stream,
                       (const K *)sorted, n, stride, count, (K *)samples);
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  });
}

extern "C" int drhip_sort_bucket_counts(int seg, int dtype, const void *sorted, size_t n,
                                        const void *splitters, int nsplit, uint64_t *counts) {
  DRHIP_GET_SEG(s, seg);
  if (!counts || nsplit < 0 || nsplit > 1023 || (n && !sorted) || (nsplit && !splitters))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort_bucket_counts: bad argument");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  return dispatch_sort_dtype(dtype, [&](auto dv) -> int {
    constexpr int DT = decltype(dv)::value;
    using U = typename KeyBits<DT>::U;
    hipLaunchKernelGGL((bucket_count_kernel<DT>), dim3(1), dim3(1024), 0, s->stream, (const U *)sorted, n,
                       (const U *)splitters, nsplit, counts);
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  });
}

namespace {
template <typename U> size_t merge_ws_bytes(size_t n, int nruns) {
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  const size_t tiles = (n + kMergeTile - 1) / kMergeTile + (size_t)nruns;
  return keys_b + ((tiles + 2 * (size_t)nruns + 2) * 8 + 255) / 256 * 256;
}
} // namespace

extern "C" int drhip_merge_workspace(int seg, int dtype, size_t n, int nruns, size_t *bytes) {
  if (!bytes || nruns < 1) return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_workspace: bad argument");
  const size_t ks = dtype_size(dtype);
  if (!ks) return set_error(DRHIP_ERR_BAD_ARG, "merge: unsupported dtype");
  *bytes = ks == 4 ? merge_ws_bytes<uint32_t>(n, nruns) : merge_ws_bytes<uint64_t>(n, nruns);
  return DRHIP_OK;
}

namespace {
// The merge-path rounds of drhip_merge_runs / drhip_merge_runs_to: the runs
// of `src` are merged pairwise, round after round, until one run is left.
// in_place (src == dst): rounds alternate between keys and tmp, and a final
// copy brings the result back when the last round ended in tmp.  Otherwise
// the rounds alternate so that the LAST one writes dst (the first reads
// src): no copy at all -- the distributed sort's all_to_all lands in src
// and the merge writes straight into the segment.
template <int DT>
int merge_rounds(Segment *s, const void *src, void *dst, size_t n, const size_t *run_offsets, int nruns, void *tmp,
                 size_t tmp_bytes) {
  using U = typename KeyBits<DT>::U;
  if (tmp_bytes < merge_ws_bytes<U>(n, nruns)) return set_error(DRHIP_ERR_BAD_ARG, "merge: workspace too small");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const bool in_place = src == dst;
  if (nruns == 1 || n <= 1) {
    if (!in_place && n) DRHIP_CHECK_HIP(hipMemcpyAsync(dst, src, n * sizeof(U), hipMemcpyDeviceToDevice, s->stream));
    return DRHIP_OK;
  }
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  unsigned long long *split = (unsigned long long *)((char *)tmp + keys_b);
  int rounds = 0;
  for (int r = nruns; r > 1; r = (r + 1) / 2) rounds++;
  U *bufs[2] = {(U *)dst, (U *)tmp};
  const U *a = (const U *)src;
  std::vector<size_t> off(run_offsets, run_offsets + nruns + 1);
  for (int k = 0; off.size() > 2; k++) {
    U *b = in_place ? bufs[(k + 1) & 1] : bufs[(rounds - 1 - k) & 1];
    MergePairs mp{};
    std::vector<size_t> next;
    unsigned tiles = 0;
    for (size_t r = 0; r + 1 < off.size(); r += 2) {
      const int p = mp.npairs++;
      const size_t a0 = off[r], amid = off[r + 1];
      const size_t end = r + 2 < off.size() ? off[r + 2] : off[r + 1];
      mp.a0[p] = a0;
      mp.alen[p] = amid - a0;
      mp.blen[p] = end - amid; // an odd last run merges with an empty B (a copy)
      mp.tile0[p] = tiles;
      tiles += (unsigned)((end - a0 + kMergeTile - 1) / kMergeTile);
      next.push_back(a0);
    }
    mp.tile0[mp.npairs] = tiles;
    next.push_back(off.back());
    const unsigned nb = tiles + (unsigned)mp.npairs;
    hipLaunchKernelGGL((merge_partition<DT>), dim3((nb + 255) / 256), dim3(256), 0, s->stream, a, mp, split);
    DRHIP_CHECK_LAUNCH();
    if (tiles) {
      hipLaunchKernelGGL((merge_tiles<DT>), dim3(tiles), dim3(kMergeThreads), 0, s->stream, a, b, mp, split);
      DRHIP_CHECK_LAUNCH();
    }
    a = b;
    off.swap(next);
  }
  if (a != (const U *)dst) DRHIP_CHECK_HIP(hipMemcpyAsync(dst, a, n * sizeof(U), hipMemcpyDeviceToDevice, s->stream));
  return DRHIP_OK;
}

int merge_check(int nruns, const size_t *run_offsets, size_t n) {
  if (nruns < 1 || !run_offsets || run_offsets[0] != 0 || run_offsets[nruns] != n)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_runs: run_offsets must go 0 .. n");
  for (int r = 0; r < nruns; r++)
    if (run_offsets[r + 1] < run_offsets[r]) return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_runs: offsets");
  if ((nruns + 1) / 2 > kMaxMergePairs) return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_merge_runs: > 128 runs");
  return DRHIP_OK;
}
} // namespace

extern "C" int drhip_merge_runs(int seg, int dtype, void *keys, size_t n, const size_t *run_offsets, int nruns,
                                void *tmp, size_t tmp_bytes) {
  DRHIP_GET_SEG(s, seg);
  if (int rc = merge_check(nruns, run_offsets, n)) return rc;
  if (nruns == 1 || n <= 1) return DRHIP_OK;
  if (!keys || !tmp || ((uintptr_t)keys & 15) || ((uintptr_t)tmp & 255))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_runs: keys 16-byte and tmp 256-byte aligned");
  return dispatch_sort_dtype(dtype, [&](auto dv) -> int {
    return merge_rounds<decltype(dv)::value>(s, keys, keys, n, run_offsets, nruns, tmp, tmp_bytes);
  });
}

extern "C" int drhip_merge_runs_to(int seg, int dtype, const void *src, void *dst, size_t n, const size_t *run_offsets,
                                   int nruns, void *tmp, size_t tmp_bytes) {
  DRHIP_GET_SEG(s, seg);
  if (int rc = merge_check(nruns, run_offsets, n)) return rc;
  if (n == 0) return DRHIP_OK;
  const size_t ks = dtype_size(dtype);
  // element-aligned src / dst suffice (merge_tiles stores 16 B only where
  // its output is 16-byte aligned): dst may be a sub-range's segment
  if (!src || !dst || !tmp || !ks || ((uintptr_t)src % ks) || ((uintptr_t)dst % ks) || ((uintptr_t)tmp & 255))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_runs_to: src / dst key-aligned and tmp 256-byte aligned");
  if (ks && ((const char *)src < (const char *)dst + n * ks && (const char *)dst < (const char *)src + n * ks) &&
      src != dst)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_merge_runs_to: src and dst overlap");
  return dispatch_sort_dtype(dtype, [&](auto dv) -> int {
    return merge_rounds<decltype(dv)::value>(s, src, dst, n, run_offsets, nruns, tmp, tmp_bytes);
  });
}
