// spmv.hip -- CSR sparse matrix-vector product and synthetic CSR generator.
//
// Replaces the gemv nonzero loop (include/dr/shp/algorithms/gemv.hpp:45-66):
// the reference launches one work-item per NONZERO, walks rowptr from row 0
// for each (csr_matrix_view.hpp:64-68, quadratic) and does an unsynchronised
// `c_v += a_v * b_v` (:62, a data race whenever two nonzeros share a row).
// Here each row is owned by a group of G lanes (CSR-vector): the group
// strides over the row's nonzeros with coalesced loads of vals/colind,
// gathers x, reduces with shuffles and one lane does y[row] += sum.
// G is picked from the average row length (nnz / m) so a ~10 nnz/row matrix
// (BASELINE config C4) uses 8-lane groups: 8 rows per wave.
// HBM bytes per launch (int32 indices, fp32): 8*nnz + 4*(m+1) + 8*m + x reads.
#include "common.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace drhip {

// threads per SpMV block (DRHIP_SPMV_BLOCK: 512 measured in round 6,
// profiles/r06ab_spmv_block512_ab.txt)
#ifndef DRHIP_SPMV_BLOCK
#define DRHIP_SPMV_BLOCK 256
#endif
constexpr int kSpmvThreads = DRHIP_SPMV_BLOCK;
// measurement knobs (tools/build_variant.sh): nontemporal colind/vals vector
// loads, nontemporal y stores
#ifndef DRHIP_SPMV_NT
#define DRHIP_SPMV_NT 0
#endif
#ifndef DRHIP_SPMV_NT_Y
#define DRHIP_SPMV_NT_Y 0
#endif

template <typename V, typename I, int G>
__global__ __launch_bounds__(kSpmvThreads) void spmv_csr_kernel(size_t m, const I *__restrict__ rowptr,
                                                               const I *__restrict__ colind,
                                                               const V *__restrict__ vals,
                                                               const V *__restrict__ x,
                                                               V *__restrict__ y) {
  const int lane_g = threadIdx.x & (G - 1);
  const size_t rows_per_grid = (size_t)gridDim.x * (kSpmvThreads / G);
  for (size_t row = (size_t)blockIdx.x * (kSpmvThreads / G) + threadIdx.x / G; row < m;
       row += rows_per_grid) {
    const I b = rowptr[row], e = rowptr[row + 1];
    V acc = V(0);
    // vals / colind are streamed once: nontemporal; x is gathered (re-read)
    for (I k = b + lane_g; k < e; k += G)
      acc += __builtin_nontemporal_load(vals + k) * x[__builtin_nontemporal_load(colind + k)];
#pragma unroll
    for (int msk = G / 2; msk >= 1; msk >>= 1) acc += shfl_xor(acc, msk);
    if (lane_g == 0) y[row] += acc;
  }
}

// CSR-stream for short rows (average <= 32 nnz): block b owns rows
// [b*RPB, (b+1)*RPB) and streams their nonzeros in chunks of NPB starting at
// the block's first nonzero rounded down to 4: every thread loads 4
// consecutive (colind, vals) per round with vector loads (VEC; 16 B for
// int32/fp32) and issues their 4 x gathers together, writes the products to
// LDS, and after a barrier each thread sums its own row's products in
// nonzero order (the oracle's order).  One owner per row, no atomics,
// deterministic.  The many independent gathers in flight per thread are what
// the x-gather-bound random matrix (BASELINE C4) needs; cached (not
// nontemporal) loads measured best (tools/spmv_sweep.hip: banded C4 1.35 ms
// vs 1.69 ms for 4-byte nontemporal loads).
#ifndef DRHIP_SPMV_MINW
#define DRHIP_SPMV_MINW 1
#endif
#ifndef DRHIP_SPMV_NPB_MAX
#define DRHIP_SPMV_NPB_MAX 2048
#endif
// One block per row block.  Two ways of taking the rowptr round trip off
// the per-block chain (rowptr -> colind/vals -> x) measured slower on banded
// C4 (tools/spmv_shapes.py, round 3): a persistent grid issuing the NEXT row
// block's bounds first (1.38-1.44 vs 1.20 ms at 4-16 blocks per CU), and
// blocks owning nonzero slots instead of rows, their rows found by a
// per-block binary search of rowptr and rows crossing a block boundary
// finished by a fixup kernel (1.249 vs 1.213 ms).  The chain's latency is not
// what bounds this kernel.
// XW > 0: LDS-cached x window of XW entries (see the VEC loop).
// DRHIP_SPMV_SPEC: the window of a one-chunk block from its first and last
// nonzero's columns, loaded without waiting for the colind vectors (1: a
// miss falls back to the block-wide min/max window; 2: a miss gathers from
// global memory, and the min/max window is compiled out -- it costs the
// 4-byte kernel its spill-free 8-wave register budget; 0: min/max only).
// Round 5, banded C4 2^26 rows, bench kernel times in three interleaved
// rounds on one box (profiles/r05_spmv_spec_ab.txt): 0 -> 1.153 / 1.129 /
// 1.157 ms, 1 -> 1.106 / 1.111 / 1.128 ms, 2 -> 1.127 / 1.168 / 1.170 ms;
// random C4 unchanged (13.38-13.49 ms in all three).
#ifndef DRHIP_SPMV_SPEC
#define DRHIP_SPMV_SPEC 1
#endif
#ifndef DRHIP_SPMV_XW
#define DRHIP_SPMV_XW 2048
#endif
// Waves per SIMD requested for the 4-byte 2048-slot kernel (the C4 shape):
// the x window's extra live registers would otherwise drop it to 5 waves
// (87 VGPRs), which measured 1.30 ms against 1.14 ms at 8 (64 VGPRs, 5
// spilled) and 1.21 ms without the window (tools/gpu_r03n.sh).
#ifndef DRHIP_SPMV_MINW_4B
#define DRHIP_SPMV_MINW_4B 8
#endif
// The window (and the 8-wave request) only for 4-byte values and indices up
// to 2048 slots, the shape measured; wider types keep the gathers from
// global memory (the window's registers would cut their occupancy).
// DRHIP_SPMV_I64_WIN (measurement knob): 8-byte indices take the window too
#ifndef DRHIP_SPMV_I64_WIN
#define DRHIP_SPMV_I64_WIN 0
#endif
template <typename V, typename I, int NPB> constexpr bool spmv_4b() {
  return sizeof(V) == 4 && (sizeof(I) == 4 || (DRHIP_SPMV_I64_WIN && sizeof(I) == 8)) && NPB <= 8 * kSpmvThreads;
}
template <typename V, typename I, int NPB> constexpr int spmv_minw() {
  return spmv_4b<V, I, NPB>() ? DRHIP_SPMV_MINW_4B : DRHIP_SPMV_MINW;
}
template <typename V, typename I, int NPB, bool VEC, int XW = (spmv_4b<V, I, NPB>() ? DRHIP_SPMV_XW : 0)>
__global__ __launch_bounds__(kSpmvThreads, (spmv_minw<V, I, NPB>())) void spmv_csr_stream_kernel(size_t m, size_t nnz,
                                                                      unsigned rpb,
                                                                      const I *__restrict__ rowptr,
                                                                      const I *__restrict__ colind,
                                                                      const V *__restrict__ vals,
                                                                      const V *__restrict__ x,
                                                                      V *__restrict__ y) {
  static_assert(NPB % (4 * kSpmvThreads) == 0, "whole rounds");
  typedef I I4 __attribute__((ext_vector_type(4)));
  typedef V V4 __attribute__((ext_vector_type(4)));
  __shared__ V4 prod4[NPB / 4];
  __shared__ V xs[XW > 0 ? XW : 1];
  __shared__ std::make_unsigned_t<I> s_cmn[kSpmvThreads / kWave], s_cmx[kSpmvThreads / kWave];
  __shared__ bool s_miss[kSpmvThreads / kWave];
  const V *prod = reinterpret_cast<const V *>(prod4);
  const int tid = threadIdx.x;
  // row block b: rows [b * rpb, + rpb), rpb <= 256 (one row per thread),
  // picked by the launcher so that a block's nonzeros fill its NPB-slot chunk
  const size_t r0 = (size_t)blockIdx.x * rpb;
  const size_t nr = m - r0 < (size_t)rpb ? m - r0 : (size_t)rpb;
  // block-uniform bounds (broadcast loads) and the thread's own row, all
  // issued up front together with the y prefetch: no barrier before the
  // first gathers
  const size_t nz0 = (size_t)rowptr[r0], nz1 = (size_t)rowptr[r0 + nr];
  const bool has_row = (size_t)tid < nr;
  const size_t rb = has_row ? (size_t)rowptr[r0 + tid] : 0, re = has_row ? (size_t)rowptr[r0 + tid + 1] : 0;
  const V y0 = has_row ? y[r0 + tid] : V(0);
  constexpr int K = NPB / (4 * kSpmvThreads);
  using UC = std::make_unsigned_t<I>;
  // Speculative x window (XW > 0): when the block's nonzeros fit ONE chunk,
  // the columns of its first and last nonzero (two broadcast loads issued
  // with the colind/vals vectors) bound the window [lo, lo + span) of a
  // banded or stencil-like block.  Every index in it is <= a column the
  // matrix holds, so the window loads are in bounds without knowing x's
  // length, and they depend on rowptr only -- not on the colind vectors
  // and a block-wide min/max as the general window below does.  Each thread
  // checks its own nonzeros against the window; one barrier publishes the
  // window and folds the checks; a miss falls back to the min/max window.
  UC sp_lo = 0, sp_span = 0;
  if constexpr (XW > 0 && VEC && DRHIP_SPMV_SPEC > 0) {
    if (nz1 > nz0 && nz1 - (nz0 & ~size_t(3)) <= (size_t)NPB && (nz0 & ~size_t(3)) + NPB <= nnz) {
      const UC cf = (UC)colind[nz0], cl = (UC)colind[nz1 - 1];
      sp_lo = cf < cl ? cf : cl;
      const UC hi = cf < cl ? cl : cf;
      sp_span = hi - sp_lo < (UC)XW ? hi - sp_lo + 1 : 0;
    }
  }
  {
    V acc = V(0);
    for (size_t c = nz0 & ~size_t(3); c < nz1; c += NPB) {
      if (VEC && c + NPB <= nnz) {
        // Branch-free: every lane loads a whole vector, so all K rounds of
        // colind/vals loads issue together, then all 4K gathers.  Vectors
        // past nz1 are redirected to the chunk's last vector (already being
        // loaded: no extra HBM bytes); entries outside [nz0, nz1) are other
        // rows' valid nonzeros whose products no row sum reads.  (A
        // per-element edge branch here serialised a second load -> gather
        // chain behind the first: tools/spmv_sweep.hip, banded C4 1.36 ->
        // 1.19 ms.)  Offsets from the block-uniform chunk base: one 32-bit
        // VGPR per vector load (SGPR base + offset), not a 64-bit address.
        const unsigned lastv = (unsigned)(((nz1 - 1) & ~size_t(3)) - c);
        const unsigned lim = (unsigned)(nz1 - c);
        const I *cb = colind + c;
        const V *vb = vals + c;
        I4 ci[K];
        V4 v[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
          unsigned o = (unsigned)(k * 4 * kSpmvThreads + 4 * tid);
          o = o < lim ? o : lastv;
#if DRHIP_SPMV_NT
          ci[k] = __builtin_nontemporal_load(reinterpret_cast<const I4 *>(cb + o));
          v[k] = __builtin_nontemporal_load(reinterpret_cast<const V4 *>(vb + o));
#else
          ci[k] = *reinterpret_cast<const I4 *>(cb + o);
          v[k] = *reinterpret_cast<const V4 *>(vb + o);
#endif
        }
        bool staged = false;
        if constexpr (XW > 0 && DRHIP_SPMV_SPEC > 0) {
          if (sp_span) {
            for (unsigned e = tid; e < (unsigned)sp_span; e += kSpmvThreads) xs[e] = x[sp_lo + e];
            // this thread's nonzeros of [nz0, nz1) (by their slot, before the
            // tail redirect) must all lie in the window
            const unsigned first = (unsigned)(nz0 - c), last = (unsigned)(nz1 - c);
            int miss = 0;
#pragma unroll
            for (int k = 0; k < K; k++) {
              const unsigned s0 = (unsigned)(k * 4 * kSpmvThreads + 4 * tid);
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const bool in = s0 + j >= first && s0 + j < last;
                miss |= in && (UC)((UC)ci[k][j] - sp_lo) >= sp_span;
              }
            }
            // one barrier publishes the window and the waves' miss flags
            // (__syncthreads_or costs three)
            const bool wmiss = __ballot(miss) != 0;
            if ((tid & (kWave - 1)) == 0) s_miss[tid / kWave] = wmiss;
            __syncthreads();
            bool any = false;
#pragma unroll
            for (int w = 0; w < kSpmvThreads / kWave; w++) any = any || s_miss[w];
            staged = !any; // block-uniform
            if (staged) {
#pragma unroll
              for (int k = 0; k < K; k++) {
                V4 p;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                  const UC e = (UC)ci[k][j] - sp_lo; // outside the window: a product no row reads
                  p[j] = v[k][j] * xs[e < sp_span ? e : 0];
                }
                prod4[k * kSpmvThreads + tid] = p;
              }
            }
          }
        }
        if constexpr (XW > 0 && DRHIP_SPMV_SPEC != 2) if (!staged) {
          // LDS-cached x window: when the chunk's columns span at most XW
          // entries (banded / stencil-like matrices), x[cmin, cmin + span)
          // is loaded once, coalesced, into LDS and the 4K gathers per
          // thread read LDS instead of issuing 4K vector-memory gathers
          UC cmn = ~UC(0), cmx = 0;
#pragma unroll
          for (int k = 0; k < K; k++) {
            const UC c0 = (UC)ci[k].x, c1 = (UC)ci[k].y, c2 = (UC)ci[k].z, c3 = (UC)ci[k].w;
            cmn = std::min(cmn, std::min(std::min(c0, c1), std::min(c2, c3)));
            cmx = std::max(cmx, std::max(std::max(c0, c1), std::max(c2, c3)));
          }
          cmn = wave_reduce<DRHIP_MIN>(cmn);
          cmx = wave_reduce<DRHIP_MAX>(cmx);
          if ((tid & (kWave - 1)) == 0) {
            s_cmn[tid / kWave] = cmn;
            s_cmx[tid / kWave] = cmx;
          }
          __syncthreads();
#pragma unroll
          for (int w = 0; w < kSpmvThreads / kWave; w++) {
            cmn = std::min(cmn, s_cmn[w]);
            cmx = std::max(cmx, s_cmx[w]);
          }
          const UC span = cmx - cmn + 1;
          staged = span <= (UC)XW; // block-uniform
          if (staged) {
            for (unsigned e = tid; e < (unsigned)span; e += kSpmvThreads) xs[e] = x[cmn + e];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < K; k++) {
              V4 p;
              p.x = v[k].x * xs[(UC)ci[k].x - cmn];
              p.y = v[k].y * xs[(UC)ci[k].y - cmn];
              p.z = v[k].z * xs[(UC)ci[k].z - cmn];
              p.w = v[k].w * xs[(UC)ci[k].w - cmn];
              prod4[k * kSpmvThreads + tid] = p;
            }
          }
        }
        if (!staged) {
#pragma unroll
          for (int k = 0; k < K; k++) {
            V4 p;
            p.x = v[k].x * x[ci[k].x];
            p.y = v[k].y * x[ci[k].y];
            p.z = v[k].z * x[ci[k].z];
            p.w = v[k].w * x[ci[k].w];
            prod4[k * kSpmvThreads + tid] = p;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; k++) {
          const size_t b = c + (size_t)k * 4 * kSpmvThreads + 4 * (size_t)tid;
          V4 p = {V(0), V(0), V(0), V(0)};
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (b + j >= nz0 && b + j < nz1) p[j] = vals[b + j] * x[colind[b + j]];
          prod4[k * kSpmvThreads + tid] = p;
        }
      }
      __syncthreads();
      const size_t lo = rb > c ? rb : c;
      const size_t hi = re < c + NPB ? re : c + NPB;
      for (size_t j = lo; j < hi; j++) acc += prod[j - c];
      __syncthreads();
    }
    if (has_row) {
#if DRHIP_SPMV_NT_Y
      __builtin_nontemporal_store(y0 + acc, y + r0 + tid);
#else
      y[r0 + tid] = y0 + acc;
#endif
    }
  }
}

// Round 6 tried a row-window form of the kernel below (x window from the
// block's rows, loaded beside rowptr: two dependent round trips instead of
// three, no spill): no gain on banded C4 (profiles/r06_spmv_rowwin_ab.txt) --
// waves wait 74 % of their cycles, but not on that chain.
template <typename V, typename I>
static int launch_spmv(Segment *s, int seg, size_t m, size_t nnz, const I *rowptr, const I *colind, const V *vals,
                       const V *x, V *y) {
  if (m == 0) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const double avg = (double)nnz / (double)m;
  auto go = [&](auto gv) -> int {
    constexpr int G = decltype(gv)::value;
    size_t rows_per_block = kSpmvThreads / G;
    size_t blocks = (m + rows_per_block - 1) / rows_per_block;
    unsigned grid = (unsigned)std::min<size_t>(blocks, (size_t)s->num_cus * 16);
    hipLaunchKernelGGL((spmv_csr_kernel<V, I, G>), dim3(grid), dim3(kSpmvThreads), 0, s->stream, m,
                       rowptr, colind, vals, x, y);
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  };
  if (avg <= 32) {
    // chunk of NPB nonzero slots (whole 256-thread x 4 rounds) and rows per
    // block rpb <= 256 chosen so the block's expected nonzeros (+ 3: the
    // chunk starts at the first nonzero rounded down to 4) FILL the chunk:
    // the largest NPB up to DRHIP_SPMV_NPB_MAX whose fill is >= 97 %, else
    // the best fill.  Banded C4 (10 nnz/row): 204 rows in 2048 slots (99.8 %)
    // instead of 256 rows in 3072 slots (83 %: every sixth lane loading a
    // redirected vector).  Larger chunks with 2-4 rows per thread (fill
    // ~100 % at 4096 / 8192 slots) measured slower, 1.21 / 1.28 vs 1.19 ms
    // (tools/spmv_shapes.py, round 3), so 2048 is the cap.
    // DRHIP_SPMV_NPB / DRHIP_SPMV_RPB override (tools/spmv sweeps).
    const int npbs[] = {1024, 2048, 3072, 4096, 8192};
    int npb_max = DRHIP_SPMV_NPB_MAX;
    if (const char *e = getenv("DRHIP_SPMV_NPB_MAX")) npb_max = atoi(e);
    int npb = 0, npb_best = 0;
    unsigned rpb = 0, rpb_best = 0;
    double best = -1;
    for (int c : npbs) {
      if (c > npb_max) break;
      if (c % (4 * kSpmvThreads)) continue; // whole rounds of the block
      const unsigned rr = (unsigned)std::max(1.0, std::min((double)kSpmvThreads, std::floor((c - 3) / (avg > 0 ? avg : 1.0))));
      const double fill = std::min(1.0, (rr * avg + 3) / c);
      if (fill >= 0.97) npb = c, rpb = rr; // the largest well-filled chunk
      if (fill > best) best = fill, npb_best = c, rpb_best = rr;
    }
    if (!npb) npb = npb_best, rpb = rpb_best;
    if (const char *e = getenv("DRHIP_SPMV_NPB")) npb = atoi(e);
    if (const char *e = getenv("DRHIP_SPMV_RPB")) rpb = (unsigned)atoi(e);
    if (rpb < 1 || rpb > (unsigned)kSpmvThreads) return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: rows per block 1..threads");
    const size_t blocks = (m + rpb - 1) / rpb;
    if (blocks > 0x7FFFFFFFull) return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: too many rows");
    const bool vec = (uintptr_t)colind % (4 * sizeof(I)) == 0 && (uintptr_t)vals % (4 * sizeof(V)) == 0;
    auto stream_go = [&](auto npbc) -> int {
      constexpr int NPB = decltype(npbc)::value;
      if constexpr (NPB % (4 * kSpmvThreads) != 0) {
        return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: DRHIP_SPMV_NPB not a whole number of block rounds");
      } else {
      auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kSpmvThreads), 0, s->stream, m, nnz, rpb, rowptr,
                           colind, vals, x, y);
      };
      if (vec) launch(spmv_csr_stream_kernel<V, I, NPB, true>);
      else launch(spmv_csr_stream_kernel<V, I, NPB, false>);
      DRHIP_CHECK_LAUNCH();
      return DRHIP_OK;
      }
    };
    switch (npb) {
    case 1024: return stream_go(std::integral_constant<int, 1024>{});
    case 2048: return stream_go(std::integral_constant<int, 2048>{});
    case 3072: return stream_go(std::integral_constant<int, 3072>{});
    case 4096: return stream_go(std::integral_constant<int, 4096>{});
    case 8192: return stream_go(std::integral_constant<int, 8192>{});
    default: return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: DRHIP_SPMV_NPB 1024/2048/3072/4096/8192");
    }
  }
  if (avg <= 4) return go(std::integral_constant<int, 4>{});
  if (avg <= 12) return go(std::integral_constant<int, 8>{});
  if (avg <= 24) return go(std::integral_constant<int, 16>{});
  if (avg <= 48) return go(std::integral_constant<int, 32>{});
  return go(std::integral_constant<int, 64>{});
}

// ---- synthetic generator: identical definitions to oracle/oracle.c ----

__host__ __device__ inline uint64_t hash3(uint64_t seed, uint64_t i, uint64_t j) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i * 0xBF58476D1CE4E5B9ull + j * 0x94D049BB133111EBull +
               0x2545F4914F6CDD1Dull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline float u01(uint64_t seed, uint64_t i, uint64_t j) {
  return (float)(hash3(seed, i, j) >> 40) * (1.0f / 16777216.0f);
}
constexpr size_t kBandLo = 4, kBandHi = 5;
__host__ __device__ inline size_t band_begin(size_t i) { return i >= kBandLo ? i - kBandLo : 0; }
__host__ __device__ inline size_t band_end(size_t i, size_t ncols) {
  size_t e = i + kBandHi + 1;
  return e < ncols ? e : ncols;
}
// nnz of rows [0, r) of the banded matrix, closed form.
__host__ __device__ inline size_t band_prefix(size_t r, size_t ncols) {
  // sum over i < r of (band_end(i) - band_begin(i)), summed piecewise
  size_t s = 0;
  // rows where the band is clipped at the start: i < kBandLo
  size_t a = r < kBandLo ? r : kBandLo;
  for (size_t i = 0; i < a; i++) {
    size_t e = band_end(i, ncols), b = band_begin(i);
    s += e > b ? e - b : 0;
  }
  if (r <= kBandLo) return s;
  // rows i in [kBandLo, r): begin = i-4, end = min(i+6, ncols)
  // unclipped rows: i + 6 <= ncols  -> 10 each
  size_t lo = kBandLo, hi = r;
  size_t unclip_hi = ncols >= kBandHi + 1 ? ncols - (kBandHi + 1) + 1 : 0; // i <= ncols-6
  size_t u_hi = hi < unclip_hi ? hi : unclip_hi;
  if (u_hi > lo) s += (u_hi - lo) * (kBandLo + kBandHi + 1);
  for (size_t i = (u_hi > lo ? u_hi : lo); i < hi; i++) {
    size_t e = band_end(i, ncols), b = band_begin(i);
    s += e > b ? e - b : 0;
  }
  return s;
}

template <typename I>
__global__ void gen_banded(size_t row0, size_t nrows, size_t ncols, uint64_t seed, size_t nnz0,
                           I *rowptr, I *colind, float *vals) {
  size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  size_t i = row0 + r;
  size_t off = band_prefix(i, ncols) - nnz0;
  rowptr[r] = (I)off;
  if (r == nrows) return;
  for (size_t c = band_begin(i); c < band_end(i, ncols); c++, off++) {
    colind[off] = (I)c;
    vals[off] = u01(seed, i, c);
  }
}

template <typename I>
__global__ void gen_random(size_t row0, size_t nrows, size_t ncols, int k, uint64_t seed, I *rowptr,
                           I *colind, float *vals) {
  size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  rowptr[r] = (I)(r * (size_t)k);
  if (r == nrows) return;
  size_t i = row0 + r;
  I *c = colind + r * (size_t)k;
  int cnt = 0;
  for (uint64_t j = 0; cnt < k; j++) {
    I cand = (I)(hash3(seed ^ 0x5bd1e995ull, i, j) % ncols);
    bool dup = false;
    for (int q = 0; q < cnt; q++) dup |= (c[q] == cand);
    if (!dup) c[cnt++] = cand;
  }
  for (int a = 1; a < k; a++) {
    I v = c[a];
    int b = a - 1;
    while (b >= 0 && c[b] > v) {
      c[b + 1] = c[b];
      b--;
    }
    c[b + 1] = v;
  }
  for (int a = 0; a < k; a++) vals[r * (size_t)k + a] = u01(seed, i, (uint64_t)c[a]);
}

// ---- density generator (sparse_matrix(shape, density), containers/
// sparse_matrix.hpp:157-166 + util/generate_random.hpp:29-90) -----------
// nnz = floor(density * m * n) as the reference computes it
// (generate_random.hpp:37), spread evenly over the m rows: row i holds
// floor((i+1) nnz / m) - floor(i nnz / m) entries.  Row i's k entries are
// one column per stratum [floor(s n / k), floor((s+1) n / k)), s < k,
// picked by hash: distinct and sorted by construction, O(k) per row (the
// reference's std::map of all entries cannot reach large matrices).  Values
// are U[0,1) floats (float/double) or hash bits in {0, 1} (integers: the
// reference's uniform_int_distribution(0, 1), generate_random.hpp:12-24).
__host__ __device__ inline size_t density_nnz_total(size_t m, size_t n, double density) {
  return (size_t)(density * (double)m * (double)n);
}
__host__ __device__ inline size_t density_prefix(size_t i, size_t m, size_t nnz) {
  return m ? (size_t)(((unsigned __int128)i * nnz) / m) : 0;
}
template <typename V> __host__ __device__ inline V density_value(uint64_t seed, size_t i, size_t c) {
  if constexpr (std::is_floating_point_v<V>) return (V)u01(seed, i, c);
  else return (V)(hash3(seed, i, c) >> 63);
}

template <typename V, typename I>
__global__ void gen_density(size_t row0, size_t nrows, size_t m, size_t ncols, size_t nnz, uint64_t seed,
                            I *rowptr, I *colind, V *vals) {
  size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  const size_t i = row0 + r;
  const size_t base = density_prefix(row0, m, nnz);
  const size_t off = density_prefix(i, m, nnz) - base;
  rowptr[r] = (I)off;
  if (r == nrows) return;
  const size_t k = density_prefix(i + 1, m, nnz) - density_prefix(i, m, nnz);
  for (size_t q = 0; q < k; q++) {
    const size_t lo = (size_t)(((unsigned __int128)q * ncols) / k);
    const size_t hi = (size_t)(((unsigned __int128)(q + 1) * ncols) / k);
    const size_t c = lo + hash3(seed ^ 0x2545F491ull, i, q) % (hi - lo);
    colind[off + q] = (I)c;
    vals[off + q] = density_value<V>(seed, i, c);
  }
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_spmv_csr(int seg, int vdtype, int idtype, size_t m, size_t nnz, const void *rowptr,
                              const void *colind, const void *vals, const void *x, void *y) {
  DRHIP_GET_SEG(s, seg);
  if (m && (!rowptr || !y || (nnz && (!colind || !vals || !x))))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: null pointer");
  if (vdtype == DRHIP_F32 && idtype == DRHIP_I32)
    return launch_spmv<float, int32_t>(s, seg, m, nnz, (const int32_t *)rowptr, (const int32_t *)colind,
                                       (const float *)vals, (const float *)x, (float *)y);
  if (vdtype == DRHIP_F32 && idtype == DRHIP_I64)
    return launch_spmv<float, int64_t>(s, seg, m, nnz, (const int64_t *)rowptr, (const int64_t *)colind,
                                       (const float *)vals, (const float *)x, (float *)y);
  if (vdtype == DRHIP_F64 && idtype == DRHIP_I32)
    return launch_spmv<double, int32_t>(s, seg, m, nnz, (const int32_t *)rowptr, (const int32_t *)colind,
                                        (const double *)vals, (const double *)x, (double *)y);
  if (vdtype == DRHIP_F64 && idtype == DRHIP_I64)
    return launch_spmv<double, int64_t>(s, seg, m, nnz, (const int64_t *)rowptr, (const int64_t *)colind,
                                        (const double *)vals, (const double *)x, (double *)y);
  return set_error(DRHIP_ERR_BAD_ARG, "drhip_spmv_csr: vdtype F32/F64, idtype I32/I64");
}

extern "C" int drhip_csr_nnz(int kind, size_t row0, size_t nrows, size_t ncols, int k, size_t *nnz) {
  if (!nnz) return set_error(DRHIP_ERR_BAD_ARG, "null");
  if (kind == 0) {
    *nnz = band_prefix(row0 + nrows, ncols) - band_prefix(row0, ncols);
  } else if (kind == 1) {
    size_t kk = (size_t)k < ncols ? (size_t)k : ncols;
    *nnz = nrows * kk;
  } else {
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_nnz: kind 0 (banded) or 1 (random)");
  }
  return DRHIP_OK;
}

extern "C" int drhip_csr_gen(int seg, int kind, size_t row0, size_t nrows, size_t ncols, int k,
                             uint64_t seed, void *rowptr, void *colind, void *vals) {
  DRHIP_GET_SEG(s, seg);
  if (!rowptr || (nrows && (!colind || !vals))) return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen: null");
  if (ncols == 0 || ncols > 0x7FFFFFFFull) return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen: ncols");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  unsigned grid = (unsigned)((nrows + 1 + 255) / 256);
  if (kind == 0) {
    size_t nnz0 = band_prefix(row0, ncols);
    hipLaunchKernelGGL((gen_banded<int32_t>), dim3(grid), dim3(256), 0, s->stream, row0, nrows, ncols, seed,
                       nnz0, (int32_t *)rowptr, (int32_t *)colind, (float *)vals);
  } else if (kind == 1) {
    int kk = (size_t)k < ncols ? k : (int)ncols;
    if (kk <= 0 || kk > 64) return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen: 1 <= k <= 64");
    hipLaunchKernelGGL((gen_random<int32_t>), dim3(grid), dim3(256), 0, s->stream, row0, nrows, ncols, kk,
                       seed, (int32_t *)rowptr, (int32_t *)colind, (float *)vals);
  } else {
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen: kind 0 (banded) or 1 (random)");
  }
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

extern "C" int drhip_csr_density_nnz(size_t row0, size_t nrows, size_t m, size_t ncols, double density,
                                     size_t *nnz) {
  if (!nnz) return set_error(DRHIP_ERR_BAD_ARG, "null");
  if (!(density >= 0.0 && density <= 1.0) || row0 + nrows > m)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_density_nnz: 0 <= density <= 1, rows within m");
  const size_t tot = density_nnz_total(m, ncols, density);
  *nnz = density_prefix(row0 + nrows, m, tot) - density_prefix(row0, m, tot);
  return DRHIP_OK;
}

extern "C" int drhip_csr_gen_density(int seg, int vdtype, int idtype, size_t row0, size_t nrows, size_t m,
                                     size_t ncols, double density, uint64_t seed, void *rowptr, void *colind,
                                     void *vals) {
  DRHIP_GET_SEG(s, seg);
  if (!(density >= 0.0 && density <= 1.0) || row0 + nrows > m)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: 0 <= density <= 1, rows within m");
  if (!rowptr || (nrows && (!colind || !vals))) return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: null");
  if (ncols == 0 || (idtype == DRHIP_I32 && (ncols > 0x7FFFFFFFull || m > 0x7FFFFFFFull)))
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: ncols");
  const size_t tot = density_nnz_total(m, ncols, density);
  if (idtype == DRHIP_I32 && density_prefix(row0 + nrows, m, tot) - density_prefix(row0, m, tot) > 0x7FFFFFFFull)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: tile nnz exceeds int32 rowptr");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const unsigned grid = (unsigned)((nrows + 1 + 255) / 256);
  auto go = [&](auto vt, auto it) -> int {
    using V = decltype(vt);
    using I = decltype(it);
    hipLaunchKernelGGL((gen_density<V, I>), dim3(grid), dim3(256), 0, s->stream, row0, nrows, m, ncols, tot, seed,
                       (I *)rowptr, (I *)colind, (V *)vals);
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  };
  auto with_i = [&](auto vt) -> int {
    if (idtype == DRHIP_I32) return go(vt, int32_t{});
    if (idtype == DRHIP_I64) return go(vt, int64_t{});
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: idtype I32/I64");
  };
  switch (vdtype) {
  case DRHIP_F32: return with_i(float{});
  case DRHIP_F64: return with_i(double{});
  case DRHIP_I32: return with_i(int32_t{});
  case DRHIP_I64: return with_i(int64_t{});
  case DRHIP_U32: return with_i(uint32_t{});
  case DRHIP_U64: return with_i(uint64_t{});
  }
  return set_error(DRHIP_ERR_BAD_ARG, "drhip_csr_gen_density: vdtype");
}
