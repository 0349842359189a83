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

namespace drhip {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kRadix = 256;
constexpr int kDigits1 = kRadix + 1; // + one slot for out-of-range lanes
#ifndef DRHIP_SORT_SUBTILES
#define DRHIP_SORT_SUBTILES 4
#endif
#ifndef DRHIP_SORT_KPL4
#define DRHIP_SORT_KPL4 16
#endif
#ifndef DRHIP_SORT_MINW
#define DRHIP_SORT_MINW 4 // tools/sort_variants.sh: 4.53 vs 4.72 ms at 2^28
#endif
constexpr int kSubTiles = DRHIP_SORT_SUBTILES; // sub-tiles per block chunk

template <typename K> struct SortCfg {
  static constexpr int KPL = sizeof(K) == 4 ? DRHIP_SORT_KPL4 : DRHIP_SORT_KPL4 / 2; // keys per lane per sub-tile
  static constexpr int SUB = kSortThreads * KPL;      // keys per sub-tile (16 KiB)
  static constexpr int CH = SUB * kSubTiles;          // keys per block chunk
  static constexpr int PASSES = (int)sizeof(K);       // 8-bit digits
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
template <int DT, bool XIN>
__global__ __launch_bounds__(kSortThreads) void radix_hist(const typename KeyBits<DT>::U *keys, size_t n,
                                                          int shift, uint32_t *hist, unsigned nblocks) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U>;
  constexpr int V = 16 / sizeof(U);
  __shared__ uint32_t s_cnt[kSortWaves][kRadix];
  const int tid = threadIdx.x, wid = tid / kWave;
  for (int i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * Cfg::CH;
  const size_t end = base + Cfg::CH < n ? base + Cfg::CH : n;
  const Vec16<U> *kv = reinterpret_cast<const Vec16<U> *>(keys);
  if (end - base == (size_t)Cfg::CH) {
    // full chunk: CH / V vectors, strided by the block
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

// -------------------------------------------------------------- scatter
template <int DT, bool XIN, bool XOUT>
__global__ __launch_bounds__(kSortThreads, DRHIP_SORT_MINW) void radix_scatter(const typename KeyBits<DT>::U *src,
                                                             typename KeyBits<DT>::U *dst, size_t n,
                                                             int shift, const uint32_t *hist,
                                                             const uint32_t *off, unsigned nblocks) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U>;
  constexpr int KPL = Cfg::KPL;
  constexpr int SUB = Cfg::SUB;
  constexpr int KPW = SUB / kSortWaves; // keys per wave per sub-tile (contiguous)

  __shared__ U s_keys[SUB];
  __shared__ uint32_t s_wcnt[kSortWaves][kDigits1]; // per-wave running counts / prefixes
  __shared__ uint32_t s_start[kDigits1];             // digit start inside the sub-tile
  __shared__ uint32_t s_sub[kDigits1];               // sub-tile digit totals
  __shared__ uint32_t s_run[kRadix];                 // global write cursor per digit
  __shared__ uint32_t s_wsum[kSortWaves];

  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const size_t base = (size_t)blockIdx.x * Cfg::CH;
  for (int d = tid; d < kRadix; d += kSortThreads) {
    const size_t h = (size_t)d * nblocks + blockIdx.x;
    s_run[d] = off[h] - hist[h];
  }
  for (int i = tid; i < kSortWaves * kDigits1; i += kSortThreads) (&s_wcnt[0][0])[i] = 0;
  __syncthreads();

  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int st = 0; st < kSubTiles; st++) {
    const size_t sbase = base + (size_t)st * SUB;
    if (sbase >= n) break; // uniform
    const unsigned valid = (unsigned)(n - sbase < (size_t)SUB ? n - sbase : (size_t)SUB);

    // ---- load: wave w owns keys [w*KPW, (w+1)*KPW) of the sub-tile, round r
    //      covers w*KPW + r*64 + lane (4-/8-byte coalesced loads)
    U key[KPL];
    uint16_t rank[KPL];
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned li = wid * KPW + r * kWave + lane;
      U k = li < valid ? __builtin_nontemporal_load(src + sbase + li) : U(0);
      if (XIN) k = KeyBits<DT>::in(k);
      key[r] = k;
    }
    // ---- stable rank inside the wave's contiguous run of keys
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned li = wid * KPW + r * kWave + lane;
      const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
      uint64_t peers = ~0ull;
#pragma unroll
      for (int b = 0; b < 9; b++) {
        const uint64_t m = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? m : ~m;
      }
      const uint32_t before = s_wcnt[wid][d];
      const unsigned below = (unsigned)__popcll(peers & lt_mask);
      rank[r] = (uint16_t)(before + below);
      // the lowest lane of each peer group advances the wave's counter
      if (below == 0) s_wcnt[wid][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // ---- per digit: prefix over waves, sub-tile total; block scan of totals
    for (int d = tid; d < kDigits1; d += kSortThreads) {
      uint32_t run = 0;
#pragma unroll
      for (int w = 0; w < kSortWaves; w++) {
        const uint32_t c = s_wcnt[w][d];
        s_wcnt[w][d] = run;
        run += c;
      }
      s_sub[d] = run;
    }
    __syncthreads();
    {
      // exclusive scan of s_sub[0..256] (257 entries): thread t scans entry t
      // (t < 256) with a DPP wave scan + LDS wave totals; entry 256 last.
      const uint32_t x = s_sub[tid];
      const uint32_t incl = wave_inclusive_scan<DRHIP_PLUS>(x);
      if (lane == kWave - 1) s_wsum[wid] = incl;
      __syncthreads();
      uint32_t wpre = 0;
#pragma unroll
      for (int w = 0; w < kSortWaves; w++) wpre += w < wid ? s_wsum[w] : 0u;
      s_start[tid] = wpre + incl - x;
      if (tid == kSortThreads - 1) s_start[kRadix] = wpre + incl;
    }
    __syncthreads();
    // ---- reorder the sub-tile by digit in LDS
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned li = wid * KPW + r * kWave + lane;
      const unsigned d = li < valid ? (unsigned)(key[r] >> shift) & 0xFF : (unsigned)kRadix;
      s_keys[s_start[d] + s_wcnt[wid][d] + rank[r]] = key[r];
    }
    __syncthreads();
    // ---- write each digit's run contiguously (valid keys occupy [0, valid))
#pragma unroll
    for (int r = 0; r < KPL; r++) {
      const unsigned p = r * kSortThreads + tid;
      if (p < valid) {
        const U k = s_keys[p];
        const unsigned d = (unsigned)(k >> shift) & 0xFF;
        dst[s_run[d] + (p - s_start[d])] = XOUT ? KeyBits<DT>::out(k) : k;
      }
    }
    __syncthreads();
    for (int d = tid; d < kRadix; d += kSortThreads) s_run[d] += s_sub[d];
    for (int i = tid; i < kSortWaves * kDigits1; i += kSortThreads) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
  }
}

// ------------------------------------------------ sample-sort helpers
template <typename K>
__global__ void sample_kernel(const K *sorted, size_t n, size_t count, K *samples) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < count) samples[i] = sorted[(size_t)(((double)i + 0.5) * (double)n / (double)count)];
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

template <int DT> static int launch_sort(Segment *s, int seg, void *keys, size_t n, void *tmp, size_t tmp_bytes);

} // namespace drhip

using namespace drhip;

namespace {

template <typename U> size_t sort_nblocks(size_t n) {
  return (n + SortCfg<U>::CH - 1) / SortCfg<U>::CH;
}

template <typename U> size_t sort_ws_bytes(size_t n) {
  const size_t nb = sort_nblocks<U>(n);
  const size_t keys_b = (n * sizeof(U) + 255) & ~size_t(255);
  const size_t hist_b = (nb * kRadix * 4 + 255) & ~size_t(255);
  return keys_b + 2 * hist_b;
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

} // namespace

template <int DT> int drhip::launch_sort(Segment *s, int seg, void *keys, size_t n, void *tmp, size_t tmp_bytes) {
  using U = typename KeyBits<DT>::U;
  using Cfg = SortCfg<U>;
  if (n <= 1) return DRHIP_OK;
  if (n >= (size_t(1) << 32)) return set_error(DRHIP_ERR_BAD_ARG, "sort: segment must hold < 2^32 keys");
  if (((uintptr_t)keys & 15) || ((uintptr_t)tmp & 255))
    return set_error(DRHIP_ERR_BAD_ARG, "sort: keys must be 16-byte and tmp 256-byte aligned");
  if (tmp_bytes < sort_ws_bytes<U>(n)) return set_error(DRHIP_ERR_BAD_ARG, "sort: workspace too small");
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
    if (first)
      hipLaunchKernelGGL((radix_hist<DT, true>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, n,
                         shift, hist, (unsigned)nb);
    else
      hipLaunchKernelGGL((radix_hist<DT, false>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, n,
                         shift, hist, (unsigned)nb);
    DRHIP_CHECK_LAUNCH();
    int rc = scan_inclusive_u32(s, seg, hist, off, nb * kRadix);
    if (rc) return rc;
#define DRHIP_SCATTER(XI, XO)                                                                          \
  hipLaunchKernelGGL((radix_scatter<DT, XI, XO>), dim3((unsigned)nb), dim3(kSortThreads), 0, s->stream, a, \
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

extern "C" int drhip_sort_sample(int seg, int dtype, const void *sorted, size_t n, size_t count,
                                 void *samples) {
  DRHIP_GET_SEG(s, seg);
  if (!count) return DRHIP_OK;
  if (!sorted || !samples || !n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_sort_sample: bad argument");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using K = decltype(tv);
    hipLaunchKernelGGL((sample_kernel<K>), dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s->stream,
                       (const K *)sorted, n, count, (K *)samples);
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
