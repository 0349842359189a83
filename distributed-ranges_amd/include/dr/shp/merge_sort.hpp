// dr/shp/merge_sort.hpp -- the general-comparator tier of shp::sort:
// a STABLE merge sort of any trivially-copyable T under any strict weak
// ordering, as HIP template kernels compiled into the caller's translation
// unit (like the user-operator reduce / scan of algorithms.hpp / scan.hpp).
//
// The reference has no sort; the contract is
// std::ranges::sort(r, comp), and this tier gives the stronger
// std::stable_sort result, so it is bit-defined and checked bit-exactly.
//
// Per segment (all segments in flight, each on its own stream):
//   1. block_sort_kernel: tiles of sort_threads * ipt<T> elements (2048
//      4-byte keys), each sorted in LDS -- every thread sorts its ipt<T>
//      consecutive items in registers (odd-even transposition, swaps only on
//      comp(b, a): stable), then log2(sort_threads) merge-path rounds inside
//      the tile;
//   2. ceil(log2(tiles)) global passes of merge_kernel, run width doubling:
//      merge_partition_kernel finds every output tile's split on the merge
//      path (one thread per tile, binary search in HBM), then every block
//      stages its tile's A and B pieces in LDS and merges them.
// The merge path takes A's element on ties (ModernGPU's lower-bound form),
// so every merge -- and the whole sort -- is stable.  HBM traffic per pass
// is one read + one write of the segment (2 * sizeof(T) B/element).  LDS
// tiles are padded (one element per ipt) and indexed with 32-bit offsets.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

namespace shp::detail::msort {

constexpr int kMsBlock = 256; // threads of a merge-pass block
// items per thread: ~32 B of keys per thread
template <typename T> constexpr int ipt() {
  return sizeof(T) <= 4 ? 8 : sizeof(T) <= 8 ? 8 : sizeof(T) <= 16 ? 4 : sizeof(T) <= 32 ? 2 : 1;
}
// LDS padding: one element after every PAD, so that the strided accesses of
// the blocked layout (thread t touches elements t*N .. t*N+N-1) and the merge
// reads near them spread over the banks (stride N+1 instead of N)
template <typename T> constexpr int pad_every() { return ipt<T>() >= 4 ? ipt<T>() : 0; }
template <typename T> constexpr std::size_t padded(std::size_t e) {
  return pad_every<T>() ? e + e / pad_every<T>() : e;
}
// threads of a block-sort block (DR_SHP_MSORT_SORT_THREADS, default 256):
// the first sorted runs are sort_threads * ipt elements long
#ifndef DR_SHP_MSORT_SORT_THREADS
#define DR_SHP_MSORT_SORT_THREADS 256
#endif
template <typename T> constexpr int sort_threads() {
  return padded<T>(std::size_t(DR_SHP_MSORT_SORT_THREADS) * ipt<T>()) * sizeof(T) <= 65536 ? DR_SHP_MSORT_SORT_THREADS
                                                                                         : kMsBlock;
}
template <typename T> constexpr std::size_t tile() { return std::size_t(kMsBlock) * ipt<T>(); }
template <typename T> constexpr std::size_t sort_tile() { return std::size_t(sort_threads<T>()) * ipt<T>(); }

// Number of A elements among the first `diag` outputs of the stable merge of
// sorted A[0, na) and B[0, nb) (A first on ties).  I: std::size_t in HBM,
// int in LDS.
template <typename I, typename PA, typename PB, typename Comp>
__host__ __device__ inline I merge_path(PA a, I na, PB b, I nb, I diag, Comp &comp) {
  I lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
  while (lo < hi) {
    const I mid = (lo + hi) / 2;
    if (!comp(b[diag - 1 - mid], a[mid])) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// A tile in LDS, indexed through the padding.
template <typename T> struct lds_view {
  T *s;
  int off;
  __device__ T &operator[](int i) const {
    const int j = off + i;
    return s[pad_every<T>() ? j + j / pad_every<T>() : j];
  }
  __device__ lds_view at(int o) const { return {s, off + o}; }
};

// Up to N outputs of the stable merge of v[ai, aend) and v[bi, bend).
template <int N, typename T, typename Comp>
__device__ inline int serial_merge(lds_view<T> v, int ai, int aend, int bi, int bend, T (&y)[N], Comp &comp) {
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
    if (ai < aend || bi < bend) {
      const bool take_b = bi < bend && (ai >= aend || comp(v[bi], v[ai]));
      if (take_b) y[k] = v[bi++];
      else y[k] = v[ai++];
      cnt = k + 1;
    }
  }
  return cnt;
}

template <typename T, std::size_t E> struct lds_tile {
  alignas(alignof(T) > 16 ? alignof(T) : 16) unsigned char raw[padded<T>(E) * sizeof(T)];
  __device__ lds_view<T> view() { return {reinterpret_cast<T *>(raw), 0}; }
};

// Step 1: every tile of `data` sorted in place.
template <typename T, typename Comp>
__global__ __launch_bounds__(sort_threads<T>()) void block_sort_kernel(T *data, std::size_t n, Comp comp) {
  constexpr int NT = sort_threads<T>();
  constexpr int N = ipt<T>();
  constexpr int TILE = (int)sort_tile<T>();
  __shared__ lds_tile<T, sort_tile<T>()> lds;
  const lds_view<T> s = lds.view();
  const std::size_t base = (std::size_t)blockIdx.x * TILE;
  const int cnt = (int)std::min<std::size_t>(TILE, n - base);
  {
    // all N loads of a thread in flight before any LDS store (a strided
    // loop of unknown trip count waits for each load in turn)
    T r[N];
#pragma unroll
    for (int k = 0; k < N; k++)
      if (k * NT + (int)threadIdx.x < cnt) r[k] = data[base + k * NT + threadIdx.x];
#pragma unroll
    for (int k = 0; k < N; k++)
      if (k * NT + (int)threadIdx.x < cnt) s[k * NT + threadIdx.x] = r[k];
  }
  __syncthreads();
  const int my = threadIdx.x * N;
  const int valid = std::max(0, std::min(N, cnt - my));
  T x[N];
#pragma unroll
  for (int k = 0; k < N; k++)
    if (k < valid) x[k] = s[my + k];
  // odd-even transposition sort of the thread's items (stable)
#pragma unroll
  for (int r = 0; r < N; r++) {
#pragma unroll
    for (int k = r & 1; k + 1 < N; k += 2)
      if (k + 1 < valid && comp(x[k + 1], x[k])) {
        const T t = x[k];
        x[k] = x[k + 1];
        x[k + 1] = t;
      }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++)
    if (k < valid) s[my + k] = x[k];
  __syncthreads();
  // merge rounds: groups of `coop` threads merge two runs of coop/2 * N
  for (int coop = 2; coop <= NT; coop *= 2) {
    const int lane = threadIdx.x % coop;
    const int g0 = (threadIdx.x / coop) * coop * N, half = coop / 2 * N;
    const int a0 = std::min(g0, cnt), a1 = std::min(g0 + half, cnt), b1 = std::min(g0 + 2 * half, cnt);
    const int na = a1 - a0, nb = b1 - a1;
    const int diag = std::min(lane * N, na + nb);
    const int i = merge_path<int>(s.at(a0), na, s.at(a1), nb, diag, comp);
    T y[N];
    const int got = serial_merge<N>(s, a0 + i, a1, a1 + diag - i, b1, y, comp);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; k++)
      if (k < got) s[a0 + diag + k] = y[k];
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < N; k++)
    if (k * NT + (int)threadIdx.x < cnt) data[base + k * NT + threadIdx.x] = s[k * NT + threadIdx.x];
}

// Geometry of one merge pass over src[0, n): pairs of sorted runs of width w
// (pair p = [2pw, 2pw + 2w)), or -- single -- the one pair A = [0, w),
// B = [w, n) of two adjacent runs of any lengths.
struct pass_geom {
  std::size_t n, w;
  bool single;
  __host__ __device__ std::size_t pair_base(std::size_t d) const { return single ? 0 : d / (2 * w) * (2 * w); }
  __host__ __device__ std::size_t pair_end(std::size_t pb) const { return single ? n : std::min(n, pb + 2 * w); }
  __host__ __device__ std::size_t na(std::size_t pb) const { return std::min(w, n - pb); }
};

// A's split of every output tile's start on its pair's merge path.
template <typename T, typename Comp>
__global__ void merge_partition_kernel(const T *src, pass_geom g, std::size_t ntiles, std::size_t *part, Comp comp) {
  const std::size_t t = (std::size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const std::size_t d = t * tile<T>();
  const std::size_t pb = g.pair_base(d), na = g.na(pb), nb = g.pair_end(pb) - pb - na;
  part[t] = merge_path<std::size_t>(src + pb, na, src + pb + na, nb, d - pb, comp);
}

template <typename T, typename Comp>
__global__ __launch_bounds__(kMsBlock) void merge_kernel(const T *src, T *dst, pass_geom g, std::size_t ntiles,
                                                         const std::size_t *part, Comp comp) {
  constexpr int N = ipt<T>();
  constexpr std::size_t TILE = tile<T>();
  __shared__ lds_tile<T, tile<T>()> lds;
  const lds_view<T> s = lds.view();
  const std::size_t t = blockIdx.x;
  const std::size_t d0 = t * TILE, pb = g.pair_base(d0), pe = g.pair_end(pb);
  const std::size_t d1 = std::min(d0 + TILE, pe);
  const std::size_t na = g.na(pb);
  const std::size_t i0 = part[t];
  const std::size_t i1 = (t + 1 < ntiles && (t + 1) * TILE < pe) ? part[t + 1] : na;
  const std::size_t j0 = (d0 - pb) - i0, j1 = (d1 - pb) - i1;
  const T *A = src + pb, *B = src + pb + na;
  const int la = (int)(i1 - i0), lb = (int)(j1 - j0);
  {
    // element e < la + lb (<= TILE) of the staged pair pieces: A's piece
    // then B's; all N loads of a thread issued before any LDS store
    T r[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
      const int e = k * kMsBlock + threadIdx.x;
      if (e < la) r[k] = A[i0 + e];
      else if (e < la + lb) r[k] = B[j0 + (e - la)];
    }
#pragma unroll
    for (int k = 0; k < N; k++) {
      const int e = k * kMsBlock + threadIdx.x;
      if (e < la + lb) s[e] = r[k];
    }
  }
  __syncthreads();
  const int diag = std::min((int)threadIdx.x * N, la + lb);
  const int i = merge_path<int>(s, la, s.at(la), lb, diag, comp);
  T y[N];
  const int got = serial_merge<N>(s, i, la, la + diag - i, la + lb, y, comp);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++)
    if (k < got) s[diag + k] = y[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++)
    if (k * kMsBlock + (int)threadIdx.x < la + lb) dst[d0 + k * kMsBlock + threadIdx.x] = s[k * kMsBlock + threadIdx.x];
}

// s[j] = data[j * stride], j < ns (the regular samples of a sorted segment).
template <typename T> __global__ void gather_samples_kernel(const T *data, std::size_t stride, std::size_t ns, T *s) {
  const std::size_t j = (std::size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < ns) s[j] = data[j * stride];
}

// Device scratch one local sort needs: a ping-pong copy of the segment and
// the tile splits.
template <typename T> constexpr std::size_t scratch_bytes(std::size_t n) {
  const std::size_t tiles = (n + tile<T>() - 1) / tile<T>();
  return ((n * sizeof(T) + 255) & ~std::size_t(255)) + (tiles + 1) * sizeof(std::size_t);
}

inline unsigned blocks_of(std::size_t n, std::size_t per) { return (unsigned)std::max<std::size_t>(1, (n + per - 1) / per); }

// One merge pass src -> dst on `st`.
template <typename T, typename Comp>
void merge_pass(const T *src, T *dst, pass_geom g, std::size_t *part, Comp comp, hipStream_t st) {
  const std::size_t ntiles = (g.n + tile<T>() - 1) / tile<T>();
  hipLaunchKernelGGL((merge_partition_kernel<T, Comp>), dim3(blocks_of(ntiles, 256)), dim3(256), 0, st, src, g,
                     ntiles, part, comp);
  hipLaunchKernelGGL((merge_kernel<T, Comp>), dim3((unsigned)ntiles), dim3(kMsBlock), 0, st, src, dst, g, ntiles,
                     part, comp);
}

// Stable sort of data[0, n) in place on stream st; scratch of
// scratch_bytes<T>(n) bytes.  Asynchronous.
template <typename T, typename Comp>
void local_sort(T *data, std::size_t n, void *scratch, Comp comp, hipStream_t st) {
  if (n <= 1) return;
  T *tmp = static_cast<T *>(scratch);
  auto *part = reinterpret_cast<std::size_t *>(static_cast<char *>(scratch) + ((n * sizeof(T) + 255) & ~std::size_t(255)));
  hipLaunchKernelGGL((block_sort_kernel<T, Comp>), dim3(blocks_of(n, sort_tile<T>())), dim3(sort_threads<T>()), 0,
                     st, data, n, comp);
  T *src = data, *dst = tmp;
  for (std::size_t w = sort_tile<T>(); w < n; w *= 2) {
    merge_pass<T>(src, dst, pass_geom{n, w, false}, part, comp, st);
    std::swap(src, dst);
  }
  if (src != data) (void)hipMemcpyAsync(data, src, n * sizeof(T), hipMemcpyDeviceToDevice, st);
}

} // namespace shp::detail::msort
