// reduce.hip -- per-segment reduction and dot product for gfx950.
//
// Replaces the oneDPL reduce_async call of shp::reduce
// (include/dr/shp/algorithms/reduce.hpp:22-34, :74-78) and the
// reduce(zip | transform(a*b)) composition of examples/shp/dot_product.cpp.
//
// Design (HBM-bound, 4 B/elem for f32):
//   stage 1: grid = min(#chunks, CUs x 8) blocks of 256 threads, each
//            owning a contiguous range; each iteration a thread issues U=8
//            independent nontemporal 16-byte loads (1 KiB per
//            wave-instruction), folds the 8xVEC elements in the element's
//            compute type (fp32 for f32 sums) and adds that into an fp64
//            (f32/f64) or wrapping-unsigned accumulator; wave butterfly + LDS
//            block reduce -> one partial per block in the workspace.
//   fold:    in the SAME kernel, the block that finishes last (a counter in
//            Segment::dsync, reset by that block) folds the partials exactly
//            as a second one-block stage would and writes the ACC result
//            (device memory, peer memory or pinned host memory): one launch
//            per reduce, no memset, replayable in a HIP graph (round 4: the
//            two-kernel form cost a second dispatch and its gap, ~6-10 us of
//            the per-rank step of strong-scaled C2).
// Misaligned heads/tails (sub-ranges) are folded by block 0 with scalar
// loads, so any T-aligned pointer works.
#include "common.hpp"

#include <type_traits>

namespace drhip {

constexpr int kReduceThreads = 256;
constexpr int kReduceU = 8;
// drhip_reduce grid: blocks per CU.  2^27 / 2^30 f32 (tools/reduce_ab.py,
// profiles/r04_reduce_grid_ab.txt, three interleaved rounds): 8 per CU
// 0.082 / 0.614 ms, 4 0.083-0.085 / 0.613, 2 0.0797 / 0.607 (7.07 TB/s).
// The dot kernel (round 5, tools/archive/r05/dot_ab.py, profiles/r05_dot_grid_ab.txt,
// 2^27 / 2^29 f32 pairs, three rounds): 8 per CU 0.159-0.164 / 0.613-0.614
// ms, 4 0.160-0.162 / 0.614-0.615, 2 0.156-0.158 / 0.606 (0.886 of 8 TB/s).
#ifndef DRHIP_REDUCE_BLOCKS_PER_CU
#define DRHIP_REDUCE_BLOCKS_PER_CU 2
#endif
constexpr int kReduceBlocksPerCU = DRHIP_REDUCE_BLOCKS_PER_CU;
#ifndef DRHIP_DOT_BLOCKS_PER_CU
#define DRHIP_DOT_BLOCKS_PER_CU 2
#endif
constexpr int kDotBlocksPerCU = DRHIP_DOT_BLOCKS_PER_CU;
constexpr int kReduceMaxBlocks = 4096;

template <int OP, typename T>
using kacc_t = std::conditional_t<std::is_floating_point_v<T>, double,
                                  typename compute_of<OP, T>::type>;
template <int OP, typename T> using kcmp_t = typename compute_of<OP, T>::type;

// Block-wide reduction of one value per thread; result valid in thread 0.
template <int OP, typename A>
__device__ __forceinline__ A block_reduce(A v, A *smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  v = wave_reduce<OP>(v);
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  if (wid == 0) {
    constexpr int nw = kReduceThreads / kWave;
    v = lane < nw ? smem[lane] : Op<OP, A>::identity();
    v = wave_reduce<OP>(v);
  }
  return v;
}

// Stage 1: block b folds the contiguous vector range [b*per, (b+1)*per)
// with kReduceU independent nontemporal 16-byte loads per thread per
// iteration (tools/reduce_sweep.hip: contiguous + nt + U = 8 is the fastest
// shape, 7.07 TB/s on 2^30 f32), folding each iteration's U x V elements in
// the element compute type before adding into the ACC accumulator.
// Thread 0 of every block stores the block's partial and counts the block
// finished; the block that counts last folds all partials (thread i takes
// partials i, i + 256, ... then the block reduce: the order of the former
// second stage, so results are bit-identical to it), writes *out and resets
// the counters for the next launch.  Hand-off (MI355X_MICROARCH "Valid
// forms"): the partial is an `sc1` (write-through) agent-scope store,
// drained by `s_waitcnt vmcnt(0)` before the relaxed counter add -- no
// release fence per block (a `buffer_wbl2` in every block made the reduce
// 2x slower at 2^27: 0.086 -> 0.183 ms); only the last block pays one agent
// acquire, then reads the partials with `sc1` loads.  The count is
// two-level -- blocks count into groups of kReduceGroup (one 128-B line per
// group counter), the last of a group into the top counter -- so no address
// takes more than max(group, groups) atomics at the kernel's end, when every
// block finishes at once.
#ifndef DRHIP_REDUCE_GROUP
#define DRHIP_REDUCE_GROUP 32
#endif
constexpr unsigned kReduceGroup = DRHIP_REDUCE_GROUP; // 0: one flat counter (measurement)
constexpr unsigned kLineWords = 32;                   // 128-B line of counters
template <int OP, typename A>
__device__ __forceinline__ void last_block_fold(A acc, A *parts, unsigned *done, A *out, A *smem) {
  __shared__ bool s_last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(parts + blockIdx.x, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool last;
    if constexpr (kReduceGroup == 0) {
      last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    } else {
      const unsigned g = blockIdx.x / kReduceGroup, ng = (gridDim.x + kReduceGroup - 1) / kReduceGroup;
      const unsigned in_g = gridDim.x - g * kReduceGroup < kReduceGroup ? gridDim.x - g * kReduceGroup : kReduceGroup;
      last = __hip_atomic_fetch_add(done + (1 + g) * kLineWords, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             in_g - 1;
      if (last) last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
    }
    s_last = last;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  A f = Op<OP, A>::identity();
  for (unsigned i = threadIdx.x; i < gridDim.x; i += kReduceThreads)
    f = Op<OP, A>::apply(f, __hip_atomic_load(parts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  f = block_reduce<OP>(f, smem);
  // reset every counter this launch used (stream order makes it visible to
  // the next launch)
  if constexpr (kReduceGroup != 0)
    for (unsigned g = threadIdx.x; g < (gridDim.x + kReduceGroup - 1) / kReduceGroup; g += kReduceThreads)
      __hip_atomic_store(done + (1 + g) * kLineWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) {
    *out = f;
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int OP, typename T>
__global__ __launch_bounds__(kReduceThreads) void reduce_stage1(
    const T *__restrict__ x, size_t head, size_t nv, size_t n, kacc_t<OP, T> *__restrict__ parts, unsigned *done,
    kacc_t<OP, T> *out) {
  using A = kacc_t<OP, T>;
  using C = kcmp_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  __shared__ A smem[kReduceThreads / kWave];
  const Vec16<T> *xv = reinterpret_cast<const Vec16<T> *>(x + head);
  const size_t per = (nv + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per < nv ? (size_t)blockIdx.x * per : nv;
  const size_t hi = lo + per < nv ? lo + per : nv;
  A acc = Op<OP, A>::identity();
  size_t i = lo + threadIdx.x;
  for (; i + (kReduceU - 1) * kReduceThreads < hi; i += (size_t)kReduceU * kReduceThreads) {
    Vec16<T> v[kReduceU];
#pragma unroll
    for (int u = 0; u < kReduceU; u++) v[u] = load_nt(xv + i + u * kReduceThreads);
    C s = Op<OP, C>::identity();
#pragma unroll
    for (int u = 0; u < kReduceU; u++)
#pragma unroll
      for (int j = 0; j < V; j++) s = Op<OP, C>::apply(s, (C)v[u].v[j]);
    acc = Op<OP, A>::apply(acc, (A)s);
  }
  for (; i < hi; i += kReduceThreads) {
    const Vec16<T> v = load_nt(xv + i);
    C s = Op<OP, C>::identity();
#pragma unroll
    for (int j = 0; j < V; j++) s = Op<OP, C>::apply(s, (C)v.v[j]);
    acc = Op<OP, A>::apply(acc, (A)s);
  }
  if (blockIdx.x == 0) {
    // scalar head [0, head) and tail [head + nv*V, n)
    size_t tail0 = head + nv * V;
    size_t nscalar = head + (n - tail0);
    for (size_t k = threadIdx.x; k < nscalar; k += kReduceThreads) {
      size_t g = k < head ? k : tail0 + (k - head);
      acc = Op<OP, A>::apply(acc, (A)(C)x[g]);
    }
  }
  acc = block_reduce<OP>(acc, smem);
  last_block_fold<OP>(acc, parts, done, out, smem);
}

// ---- dot: sum x[i]*y[i] (same shape, two nontemporal streams) -----------

// y element loads of vector slot i: one 16-byte load when y shares x's
// alignment, else V nontemporal element loads (a zipped pair of shifted
// sub-ranges such as dot(x[1:], y[:-1])); the lanes of a wave still read
// consecutive 16-byte runs, so the scalar form stays fully coalesced.
template <bool YVEC, typename T>
__device__ __forceinline__ Vec16<T> load_y(const T *__restrict__ y, size_t i) {
  if constexpr (YVEC) {
    return load_nt(reinterpret_cast<const Vec16<T> *>(y) + i);
  } else {
    Vec16<T> r;
#pragma unroll
    for (int j = 0; j < Vec16<T>::N; j++) r.v[j] = __builtin_nontemporal_load(y + i * Vec16<T>::N + j);
    return r;
  }
}

template <typename T, bool YVEC>
__global__ __launch_bounds__(kReduceThreads) void dot_stage1(const T *__restrict__ x,
                                                            const T *__restrict__ y, size_t head,
                                                            size_t nv, size_t n,
                                                            kacc_t<DRHIP_PLUS, T> *__restrict__ parts,
                                                            unsigned *done, kacc_t<DRHIP_PLUS, T> *out) {
  using A = kacc_t<DRHIP_PLUS, T>;
  using C = kcmp_t<DRHIP_PLUS, T>;
  constexpr int V = Vec16<T>::N;
  constexpr int U = kReduceU / 2;
  __shared__ A smem[kReduceThreads / kWave];
  const Vec16<T> *xv = reinterpret_cast<const Vec16<T> *>(x + head);
  const T *yh = y + head;
  const size_t per = (nv + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per < nv ? (size_t)blockIdx.x * per : nv;
  const size_t hi = lo + per < nv ? lo + per : nv;
  A acc = A(0);
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * kReduceThreads < hi; i += (size_t)U * kReduceThreads) {
    Vec16<T> a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      a[u] = load_nt(xv + i + u * kReduceThreads);
      b[u] = load_y<YVEC>(yh, i + u * kReduceThreads);
    }
    C s = C(0);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) s += (C)a[u].v[j] * (C)b[u].v[j];
    acc += (A)s;
  }
  for (; i < hi; i += kReduceThreads) {
    const Vec16<T> a = load_nt(xv + i), b = load_y<YVEC>(yh, i);
    C s = C(0);
#pragma unroll
    for (int j = 0; j < V; j++) s += (C)a.v[j] * (C)b.v[j];
    acc += (A)s;
  }
  if (blockIdx.x == 0) {
    size_t tail0 = head + nv * V;
    size_t nscalar = head + (n - tail0);
    for (size_t k = threadIdx.x; k < nscalar; k += kReduceThreads) {
      size_t g = k < head ? k : tail0 + (k - head);
      acc += (A)((C)x[g] * (C)y[g]);
    }
  }
  acc = block_reduce<DRHIP_PLUS>(acc, smem);
  last_block_fold<DRHIP_PLUS>(acc, parts, done, out, smem);
}

// Elements before the first 16-byte boundary.
template <typename T> static size_t align_head(const void *p, size_t n) {
  uintptr_t a = (uintptr_t)p;
  size_t mis = (a & 15) ? (16 - (a & 15)) / sizeof(T) : 0;
  return mis < n ? mis : n;
}

template <typename T, int OP>
static int launch_reduce(Segment *s, int seg, const T *x, size_t n, void *out) {
  using A = kacc_t<OP, T>;
  constexpr int V = Vec16<T>::N;
  size_t head = align_head<T>(x, n);
  size_t nv = (n - head) / V;
  size_t chunks = (nv + (size_t)kReduceThreads * kReduceU - 1) / ((size_t)kReduceThreads * kReduceU);
  unsigned grid = (unsigned)std::min<size_t>(std::max<size_t>(chunks, 1),
                                             std::min<unsigned>(grid_cap(s, kReduceBlocksPerCU), kReduceMaxBlocks));
  int rc = ensure_workspace(seg, grid * sizeof(A));
  if (rc) return rc;
  A *parts = (A *)s->ws;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  hipLaunchKernelGGL((reduce_stage1<OP, T>), dim3(grid), dim3(kReduceThreads), 0, s->stream, x, head,
                     nv, n, parts, s->dsync + kSyncReduce, (A *)out);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

template <typename T>
static int launch_dot(Segment *s, int seg, const T *x, const T *y, size_t n, void *out) {
  using A = kacc_t<DRHIP_PLUS, T>;
  constexpr int V = Vec16<T>::N;
  size_t head = align_head<T>(x, n);
  // x drives the 16-byte slots; y is read with vector loads when it shares
  // x's alignment and element loads otherwise (multi-block either way).
  const bool yvec = align_head<T>(y, n) == head;
  size_t nv = (n - head) / V;
  size_t blocks = (nv + (size_t)kReduceThreads * kReduceU - 1) / ((size_t)kReduceThreads * kReduceU);
  unsigned grid = (unsigned)std::min<size_t>(std::max<size_t>(blocks, 1),
                                             std::min<unsigned>(grid_cap(s, kDotBlocksPerCU), kReduceMaxBlocks));
  int rc = ensure_workspace(seg, grid * sizeof(A));
  if (rc) return rc;
  A *parts = (A *)s->ws;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (yvec)
    hipLaunchKernelGGL((dot_stage1<T, true>), dim3(grid), dim3(kReduceThreads), 0, s->stream, x, y, head, nv, n,
                       parts, s->dsync + kSyncDot, (A *)out);
  else
    hipLaunchKernelGGL((dot_stage1<T, false>), dim3(grid), dim3(kReduceThreads), 0, s->stream, x, y, head, nv,
                       n, parts, s->dsync + kSyncDot, (A *)out);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

// The combine of shp::reduce / inclusive_scan over gathered segment results
// (reduce.hpp:81-83 host fold in segment order; inclusive_scan.hpp:108-116
// the scan of the partials): ONE thread folds the w values left to right,
// so float partials combine in exactly the reference's order.
template <int OP, typename T>
__global__ void fold_partials_kernel(const T *p, int w, int rank, T *res, T *carry) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  using C = typename compute_of<OP, T>::type;
  C acc = (C)p[0];
  for (int k = 1; k < w; k++) {
    if (k == rank && carry) *carry = (T)acc;
    acc = Op<OP, C>::apply(acc, (C)p[k]);
  }
  if (res) *res = (T)acc;
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_fold_partials(int seg, int dtype, int op, const void *partials, int w, int rank, void *result,
                                   void *carry) {
  DRHIP_GET_SEG(s, seg);
  if (!partials || w < 1 || rank < 0 || rank >= w) return set_error(DRHIP_ERR_BAD_ARG, "drhip_fold_partials: args");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      hipLaunchKernelGGL((fold_partials_kernel<OP, T>), dim3(1), dim3(64), 0, s->stream, (const T *)partials, w, rank,
                         (T *)result, (T *)carry);
      DRHIP_CHECK_LAUNCH();
      return DRHIP_OK;
    });
  });
}

extern "C" int drhip_reduce(int seg, int dtype, int op, const void *x, size_t n, void *out_acc) {
  DRHIP_GET_SEG(s, seg);
  if (!out_acc || (!x && n)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_reduce: null pointer");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      return launch_reduce<T, OP>(s, seg, (const T *)x, n, out_acc);
    });
  });
}

extern "C" int drhip_dot(int seg, int dtype, const void *x, const void *y, size_t n, void *out_acc) {
  DRHIP_GET_SEG(s, seg);
  if (!out_acc || ((!x || !y) && n)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_dot: null pointer");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return launch_dot<T>(s, seg, (const T *)x, (const T *)y, n, out_acc);
  });
}
