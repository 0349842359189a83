// dr/shp/algorithms.hpp -- shp algorithms over distributed ranges.
//
// for_each      shp/algorithms/for_each.hpp:14-92
// reduce        shp/algorithms/reduce.hpp:20-124 (6 overloads)
// transform_reduce / dot  (examples/shp/dot_product.cpp:11-18 composition)
// inclusive_scan shp/algorithms/inclusive_scan.hpp:22-218 (6 overloads)
// exclusive_scan, fill, iota, copy (shp/copy.hpp:19-173), sort (new; the
// reference has none)
//
// Standard operators (std::plus / std::multiplies / shp::minimum /
// shp::maximum) over contiguous segments of arithmetic types dispatch to
// the hand-written gfx950 kernels of libdrhip.so through the C-ABI.  Any
// other callable runs through the HIP template kernels below, compiled into
// the caller's translation unit by hipcc (the reference compiles user
// lambdas with the SYCL compiler the same way).  Callables must be
// device-callable: lambdas are; named functors need __host__ __device__ (or
// constexpr) call operators.  Every algorithm blocks until its work on all
// segments is done, like the reference.
#pragma once

#include <algorithm>
#include <cstring>
#include <memory>
#include <functional>
#include <optional>
#include <type_traits>

#include "ranges.hpp"
#include "scan.hpp"

namespace shp {

// std::ranges::min/max as device-callable function objects for reduce/scan.
template <typename T = void> struct minimum {
  __host__ __device__ constexpr auto operator()(const auto &a, const auto &b) const { return b < a ? b : a; }
};
template <typename T = void> struct maximum {
  __host__ __device__ constexpr auto operator()(const auto &a, const auto &b) const { return a < b ? b : a; }
};

namespace detail {

constexpr int kThreads = 256;

template <typename T> constexpr int dtype_code() {
  if constexpr (std::is_same_v<T, std::int32_t>) return DRHIP_I32;
  else if constexpr (std::is_same_v<T, std::uint32_t>) return DRHIP_U32;
  else if constexpr (std::is_same_v<T, std::int64_t> || (std::is_same_v<T, long long> && sizeof(long long) == 8))
    return DRHIP_I64;
  else if constexpr (std::is_same_v<T, std::uint64_t> ||
                     (std::is_same_v<T, unsigned long long> && sizeof(unsigned long long) == 8))
    return DRHIP_U64;
  else if constexpr (std::is_same_v<T, float>) return DRHIP_F32;
  else if constexpr (std::is_same_v<T, double>) return DRHIP_F64;
  else return -1;
}
template <typename T> constexpr bool abi_type = dtype_code<std::remove_cv_t<T>>() >= 0;
// ACC of the C-ABI: double for floating point, the type itself otherwise.
template <typename T> using abi_acc_t = std::conditional_t<std::is_floating_point_v<T>, double, T>;

template <typename Op> constexpr int op_code() {
  using O = std::remove_cvref_t<Op>;
  if constexpr (std::is_same_v<O, std::plus<>> || requires { requires std::is_same_v<O, std::plus<typename O::first_argument_type>>; })
    return DRHIP_PLUS;
  else if constexpr (std::is_same_v<O, std::multiplies<>> ||
                     requires { requires std::is_same_v<O, std::multiplies<typename O::first_argument_type>>; })
    return DRHIP_MUL;
  else if constexpr (std::is_same_v<O, minimum<>>) return DRHIP_MIN;
  else if constexpr (std::is_same_v<O, maximum<>>) return DRHIP_MAX;
  else return -1;
}


// One block per chunk of `per_block` items (no grid-stride residency cap):
// streaming kernels measured faster with one-shot grids (csrc/elementwise.hip).
inline int gridsize_oneshot(std::size_t n, std::size_t per_block) {
  const std::size_t g = (n + per_block - 1) / per_block;
  return static_cast<int>(std::min<std::size_t>(std::max<std::size_t>(g, 1), std::size_t(1) << 30));
}
inline int gridsize(std::size_t n) {
  std::size_t g = (n + kThreads - 1) / kThreads;
  return static_cast<int>(std::min<std::size_t>(std::max<std::size_t>(g, 1), 256 * 8));
}

// Pinned, device-visible scalars (one per segment) for C-ABI results: the
// kernels write them directly, the host reads them after the stream sync.
template <typename A> class pinned {
public:
  explicit pinned(std::size_t n) {
    p_ = static_cast<A *>(host_pool().get(std::max<std::size_t>(n, 1) * sizeof(A), cap_));
  }
  ~pinned() { host_pool().put(p_, cap_); }
  pinned(const pinned &) = delete;
  A *data() { return p_; }
  A &operator[](std::size_t i) { return p_[i]; }

private:
  A *p_ = nullptr;
  std::size_t cap_ = 0;
};

// ---------------------------------------------------------- HIP kernels

// Each block walks chunks of kForEachUnroll * kThreads elements; a thread
// calls fn on U elements kThreads apart, so for accessors whose addresses
// are base + i the U loads of a chunk are provably distinct and issue
// together (one load in flight per wave left the kernel latency-bound at
// ~54 % of HBM).
#ifndef DRHIP_FOREACH_UNROLL
#define DRHIP_FOREACH_UNROLL 8
#endif
constexpr int kForEachUnroll = DRHIP_FOREACH_UNROLL;
#ifndef DRHIP_FOREACH_STAGED_UNROLL
#define DRHIP_FOREACH_STAGED_UNROLL 1
#endif
constexpr int kForEachStagedUnroll = DRHIP_FOREACH_STAGED_UNROLL;
#ifndef DRHIP_REDUCE_UNROLL
#define DRHIP_REDUCE_UNROLL 4
#endif
constexpr int kReduceUnroll = DRHIP_REDUCE_UNROLL;
#ifndef DRHIP_REDUCE_BLOCKS
#define DRHIP_REDUCE_BLOCKS 2048
#endif
// (round 5: E consecutive elements per thread per unroll step, to let the
// compiler merge a functor's element accesses, measured no gain over this
// form -- profiles/r05_foreach_blk_ab.txt)
template <typename Acc, typename F>
__global__ __launch_bounds__(kThreads) void for_each_kernel(Acc a, std::size_t n, F f) {
  constexpr int U = kForEachUnroll;
  constexpr std::size_t chunk = (std::size_t)kThreads * U;
  const std::size_t stride = (std::size_t)gridDim.x * chunk;
  std::size_t base = blockIdx.x * chunk;
  for (; base + chunk <= n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; u++) f(a(base + (std::size_t)u * kThreads + threadIdx.x));
  }
  if (base < n) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const std::size_t i = base + (std::size_t)u * kThreads + threadIdx.x;
      if (i < n) f(a(i));
    }
  }
}

// Staged for_each over a contiguous segment (element i at base + i) of a
// trivially copyable T: each lane loads 16-byte groups of 16/sizeof(T)
// consecutive elements (U groups kThreads apart in flight), runs fn on
// register copies and writes a group back only if fn changed its bits.  fn
// sees each element exactly once, as in the reference's per-element
// parallel_for (for_each.hpp:30-46); what it cannot do here is reach other
// elements through the address of its argument.  Elements past the last
// whole group run in place.
template <typename T, typename Acc, typename F>
__global__ __launch_bounds__(kThreads) void for_each_staged_kernel(T *p, Acc a, std::size_t n, F f) {
  constexpr int V = 16 / sizeof(T);
  constexpr int U = kForEachStagedUnroll;
  typedef unsigned int W __attribute__((ext_vector_type(4)));
  const std::size_t nv = n / V;
  const std::size_t chunk = (std::size_t)kThreads * U;
  const std::size_t stride = (std::size_t)gridDim.x * chunk;
  W *pw = reinterpret_cast<W *>(p);
  auto apply = [&](std::size_t g, W &w) {
    T t[V];
    __builtin_memcpy(t, &w, 16);
#pragma unroll
    for (int k = 0; k < V; k++) f(a.bind(g * V + k, t[k]));
    W o;
    __builtin_memcpy(&o, t, 16);
    if (o.x != w.x || o.y != w.y || o.z != w.z || o.w != w.w) __builtin_nontemporal_store(o, pw + g);
  };
  std::size_t base = blockIdx.x * chunk;
  for (; base + chunk <= nv; base += stride) {
    W w[U];
#pragma unroll
    for (int u = 0; u < U; u++) w[u] = __builtin_nontemporal_load(pw + base + u * kThreads + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; u++) apply(base + u * kThreads + threadIdx.x, w[u]);
  }
  if (base < nv) {
    for (int u = 0; u < U; u++) {
      const std::size_t g = base + u * kThreads + threadIdx.x;
      if (g < nv) {
        W w = __builtin_nontemporal_load(pw + g);
        apply(g, w);
      }
    }
  }
  if (blockIdx.x == 0)
    for (std::size_t i = nv * V + threadIdx.x; i < n; i += kThreads) f(a.bind(i, p[i]));
}

// (enumerate / zip(iota, span) is NOT staged: its typical functor only
// writes the element, 4 B/elem with the plain kernel, and a staged kernel
// would read it too.  Measured on dense_bench's enumerate op, whose values
// repeat every call, the staged kernel skipped every store and looked
// faster; the write-only traffic is the honest comparison.)
// Staged for_each over zip(a, b) of two contiguous spans with elements of
// one size: 16-byte nontemporal groups of both spans, fn on the zip
// accessor's tuple of references bound to register copies, each group
// written back only if fn changed its bits (never for a const span).  The
// contract of for_each_staged_kernel: fn sees each element pair once and
// does not reach other elements through its argument's addresses.
template <typename T1, typename T2, typename F>
__global__ __launch_bounds__(kThreads) void for_each_zip2_staged_kernel(T1 *p1, T2 *p2, std::size_t n, F f) {
  static_assert(sizeof(T1) == sizeof(T2), "one group width for both spans");
  using M1 = std::remove_const_t<T1>;
  using M2 = std::remove_const_t<T2>;
  constexpr int V = 16 / sizeof(T1);
  typedef unsigned int W __attribute__((ext_vector_type(4)));
  const std::size_t nv = n / V;
  auto apply = [&](std::size_t g) {
    const W w1 = __builtin_nontemporal_load(reinterpret_cast<const W *>(p1) + g);
    const W w2 = __builtin_nontemporal_load(reinterpret_cast<const W *>(p2) + g);
    M1 a[V];
    M2 b[V];
    __builtin_memcpy(a, &w1, 16);
    __builtin_memcpy(b, &w2, 16);
#pragma unroll
    for (int k = 0; k < V; k++) f(std::tuple<T1 &, T2 &>(a[k], b[k]));
    W o1, o2;
    __builtin_memcpy(&o1, a, 16);
    __builtin_memcpy(&o2, b, 16);
    if constexpr (!std::is_const_v<T1>)
      if (o1.x != w1.x || o1.y != w1.y || o1.z != w1.z || o1.w != w1.w)
        __builtin_nontemporal_store(o1, reinterpret_cast<W *>(p1) + g);
    if constexpr (!std::is_const_v<T2>)
      if (o2.x != w2.x || o2.y != w2.y || o2.z != w2.z || o2.w != w2.w)
        __builtin_nontemporal_store(o2, reinterpret_cast<W *>(p2) + g);
  };
  const std::size_t g = (std::size_t)blockIdx.x * kThreads + threadIdx.x;
  if (g < nv) apply(g);
  if (blockIdx.x == 0)
    for (std::size_t i = nv * V + threadIdx.x; i < n; i += kThreads) f(std::tuple<T1 &, T2 &>(p1[i], p2[i]));
}

template <typename A> struct zip2_spans : std::false_type {};
template <typename T1, typename T2> struct zip2_spans<zip_accessor<span_accessor<T1>, span_accessor<T2>>> : std::true_type {
  using E1 = T1;
  using E2 = T2;
};

template <typename Seg> auto value_type_of_segment() {
  using Acc = decltype(accessor_of(std::declval<Seg>()));
  using R = decltype(std::declval<Acc>()(std::size_t(0)));
  return std::type_identity<std::remove_cvref_t<R>>{};
}

template <typename T> struct maybe {
  T v;
  bool ok;
};

// Generic reduction without an identity: per-thread fold of its strided
// elements, then an LDS tree over the valid partials; block result to
// part[blockIdx.x].
template <typename T, typename Acc, typename Op>
__global__ __launch_bounds__(kThreads) void generic_reduce_kernel(Acc a, std::size_t n, Op op, maybe<T> *part) {
  __shared__ T sv[kThreads];
  __shared__ bool sk[kThreads];
  T acc{};
  bool ok = false;
  // chunks of kReduceUnroll * kThreads: a thread's U loads are independent of
  // its running fold, so they issue together (one load in flight per wave
  // left this kernel latency-bound)
  constexpr int U = kReduceUnroll;
  constexpr std::size_t chunk = (std::size_t)kThreads * U;
  std::size_t base = blockIdx.x * chunk;
  for (; base + chunk <= n; base += (std::size_t)gridDim.x * chunk) {
    T x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = static_cast<T>(a(base + u * kThreads + threadIdx.x));
    acc = ok ? static_cast<T>(op(acc, x[0])) : x[0];
    ok = true;
#pragma unroll
    for (int u = 1; u < U; u++) acc = static_cast<T>(op(acc, x[u]));
  }
  if (base < n) {
    for (int u = 0; u < U; u++) {
      const std::size_t i = base + u * kThreads + threadIdx.x;
      if (i < n) {
        T x = static_cast<T>(a(i));
        acc = ok ? static_cast<T>(op(acc, x)) : x;
        ok = true;
      }
    }
  }
  sv[threadIdx.x] = acc;
  sk[threadIdx.x] = ok;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s && sk[threadIdx.x + s]) {
      sv[threadIdx.x] = sk[threadIdx.x] ? static_cast<T>(op(sv[threadIdx.x], sv[threadIdx.x + s]))
                                        : sv[threadIdx.x + s];
      sk[threadIdx.x] = true;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = {sv[0], sk[0]};
}

// Generic reduction over a contiguous segment (device_span) of a trivially
// copyable T: 16-byte nontemporal groups of 16/sizeof(T) elements, U groups
// kThreads apart in flight per thread, folded in registers; the elements
// past the last whole group are folded by block 0.  Same output contract as
// generic_reduce_kernel.
template <typename T, typename E, typename Op>
__global__ __launch_bounds__(kThreads) void generic_reduce_staged_kernel(const E *p, std::size_t n, Op op,
                                                                         maybe<T> *part) {
  __shared__ T sv[kThreads];
  __shared__ bool sk[kThreads];
  constexpr int V = 16 / sizeof(E);
  constexpr int U = kReduceUnroll;
  typedef unsigned int W __attribute__((ext_vector_type(4)));
  const W *pw = reinterpret_cast<const W *>(p);
  const std::size_t nv = n / V;
  constexpr std::size_t chunk = (std::size_t)kThreads * U;
  T acc{};
  bool ok = false;
  auto fold = [&](const W &w) {
    E e[V];
    __builtin_memcpy(e, &w, 16);
    acc = ok ? static_cast<T>(op(acc, static_cast<T>(e[0]))) : static_cast<T>(e[0]);
    ok = true;
#pragma unroll
    for (int k = 1; k < V; k++) acc = static_cast<T>(op(acc, static_cast<T>(e[k])));
  };
  std::size_t base = blockIdx.x * chunk;
  for (; base + chunk <= nv; base += (std::size_t)gridDim.x * chunk) {
    W w[U];
#pragma unroll
    for (int u = 0; u < U; u++) w[u] = __builtin_nontemporal_load(pw + base + u * kThreads + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; u++) fold(w[u]);
  }
  if (base < nv)
    for (int u = 0; u < U; u++) {
      const std::size_t g = base + u * kThreads + threadIdx.x;
      if (g < nv) fold(__builtin_nontemporal_load(pw + g));
    }
  if (blockIdx.x == 0)
    for (std::size_t i = nv * V + threadIdx.x; i < n; i += kThreads) {
      acc = ok ? static_cast<T>(op(acc, static_cast<T>(p[i]))) : static_cast<T>(p[i]);
      ok = true;
    }
  sv[threadIdx.x] = acc;
  sk[threadIdx.x] = ok;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s && sk[threadIdx.x + s]) {
      sv[threadIdx.x] = sk[threadIdx.x] ? static_cast<T>(op(sv[threadIdx.x], sv[threadIdx.x + s]))
                                        : sv[threadIdx.x + s];
      sk[threadIdx.x] = true;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = {sv[0], sk[0]};
}

// Generic reduction of transform(zip(a, b), f) over two contiguous segments
// (the reference's dot composition, examples/shp/dot_product.cpp:11-18) with
// elements of one size: 16-byte nontemporal groups of BOTH spans, U groups
// in flight per thread, f applied to each pair of register copies (as the
// zip accessor's tuple of references), folded with op.  Same contract as
// generic_reduce_kernel.
template <typename T, typename E1, typename E2, typename F, typename Op>
__global__ __launch_bounds__(kThreads) void generic_reduce_zip2_kernel(const E1 *p1, const E2 *p2, std::size_t n,
                                                                       F f, Op op, maybe<T> *part) {
  static_assert(sizeof(E1) == sizeof(E2), "one group width for both spans");
  __shared__ T sv[kThreads];
  __shared__ bool sk[kThreads];
  constexpr int V = 16 / sizeof(E1);
  constexpr int U = kReduceUnroll;
  typedef unsigned int W __attribute__((ext_vector_type(4)));
  const W *w1p = reinterpret_cast<const W *>(p1);
  const W *w2p = reinterpret_cast<const W *>(p2);
  const std::size_t nv = n / V;
  constexpr std::size_t chunk = (std::size_t)kThreads * U;
  T acc{};
  bool ok = false;
  auto fold1 = [&](E1 a, E2 b) {
    const T t = static_cast<T>(f(std::tuple<E1 &, E2 &>(a, b)));
    acc = ok ? static_cast<T>(op(acc, t)) : t;
    ok = true;
  };
  auto fold = [&](const W &x1, const W &x2) {
    E1 a[V];
    E2 b[V];
    __builtin_memcpy(a, &x1, 16);
    __builtin_memcpy(b, &x2, 16);
#pragma unroll
    for (int k = 0; k < V; k++) fold1(a[k], b[k]);
  };
  std::size_t base = blockIdx.x * chunk;
  for (; base + chunk <= nv; base += (std::size_t)gridDim.x * chunk) {
    W x1[U], x2[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      x1[u] = __builtin_nontemporal_load(w1p + base + u * kThreads + threadIdx.x);
      x2[u] = __builtin_nontemporal_load(w2p + base + u * kThreads + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; u++) fold(x1[u], x2[u]);
  }
  if (base < nv)
    for (int u = 0; u < U; u++) {
      const std::size_t g = base + u * kThreads + threadIdx.x;
      if (g < nv) fold(__builtin_nontemporal_load(w1p + g), __builtin_nontemporal_load(w2p + g));
    }
  if (blockIdx.x == 0)
    for (std::size_t i = nv * V + threadIdx.x; i < n; i += kThreads) fold1(p1[i], p2[i]);
  sv[threadIdx.x] = acc;
  sk[threadIdx.x] = ok;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s && sk[threadIdx.x + s]) {
      sv[threadIdx.x] = sk[threadIdx.x] ? static_cast<T>(op(sv[threadIdx.x], sv[threadIdx.x + s]))
                                        : sv[threadIdx.x + s];
      sk[threadIdx.x] = true;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = {sv[0], sk[0]};
}

template <typename S> struct zip2_transform : std::false_type {};
template <typename T1, typename L1, typename T2, typename L2, typename F>
struct zip2_transform<transform_segment<zip_segment<device_span<T1, L1>, device_span<T2, L2>>, F>> : std::true_type {
  using E1 = std::remove_const_t<T1>;
  using E2 = std::remove_const_t<T2>;
};

// Launch the generic reduction of one segment into part[0..grid).
template <typename V, typename S, typename Op> void launch_generic_reduce(const S &s, Op op, int grid, maybe<V> *part) {
  if constexpr (zip2_transform<S>::value) {
    using E1 = typename zip2_transform<S>::E1;
    using E2 = typename zip2_transform<S>::E2;
    if constexpr (std::is_trivially_copyable_v<E1> && std::is_trivially_copyable_v<E2> && sizeof(E1) == sizeof(E2) &&
                  16 % sizeof(E1) == 0) {
      const auto *p1 = std::get<0>(s.base.parts).data();
      const auto *p2 = std::get<1>(s.base.parts).data();
      if (reinterpret_cast<std::uintptr_t>(p1) % 16 == 0 && reinterpret_cast<std::uintptr_t>(p2) % 16 == 0) {
        hipLaunchKernelGGL((generic_reduce_zip2_kernel<V, E1, E2, decltype(s.f), Op>), dim3(grid), dim3(kThreads), 0,
                           stream(s.rank()), static_cast<const E1 *>(p1), static_cast<const E2 *>(p2), s.size(),
                           s.f, op, part);
        hip_check(hipGetLastError(), "reduce launch");
        return;
      }
    }
  }
  if constexpr (is_device_span<S>) {
    using E = std::remove_const_t<typename S::value_type>;
    if constexpr (std::is_trivially_copyable_v<E> && 16 % sizeof(E) == 0) {
      if (reinterpret_cast<std::uintptr_t>(s.data()) % 16 == 0) {
        hipLaunchKernelGGL((generic_reduce_staged_kernel<V, E, Op>), dim3(grid), dim3(kThreads), 0, stream(s.rank()),
                           static_cast<const E *>(s.data()), s.size(), op, part);
        hip_check(hipGetLastError(), "reduce launch");
        return;
      }
    }
  }
  auto a = accessor_of(s);
  hipLaunchKernelGGL((generic_reduce_kernel<V, decltype(a), Op>), dim3(grid), dim3(kThreads), 0, stream(s.rank()), a,
                     s.size(), op, part);
  hip_check(hipGetLastError(), "reduce launch");
}

template <typename F> void each_segment(auto &&segs, F &&f) {
  std::vector<std::size_t> ranks;
  for (auto &&s : segs) {
    if (s.size() == 0) continue;
    f(s);
    ranks.push_back(s.rank());
  }
  std::sort(ranks.begin(), ranks.end());
  ranks.erase(std::unique(ranks.begin(), ranks.end()), ranks.end());
  for (auto r : ranks) sync(r);
}

} // namespace detail

// ---------------------------------------------------------------- for_each
// for_each.hpp:14-92: fn(element) for every element of every segment.
template <typename ExecutionPolicy, typename R, typename Fn>
  requires lib::distributed_range<R>
void for_each(ExecutionPolicy &&, R &&r, Fn fn) {
  auto launch = [&](auto a, const auto &s) {
    using A = decltype(a);
    if constexpr (detail::zip2_spans<A>::value) {
      using T1 = typename detail::zip2_spans<A>::E1;
      using T2 = typename detail::zip2_spans<A>::E2;
      if constexpr (std::is_trivially_copyable_v<T1> && std::is_trivially_copyable_v<T2> && sizeof(T1) == sizeof(T2) &&
                    16 % sizeof(T1) == 0) {
        T1 *p1 = std::get<0>(a.a).p;
        T2 *p2 = std::get<1>(a.a).p;
        // overlapping spans keep the plain kernel: register copies would
        // break the aliasing the functor sees through its two references
        const auto b1 = reinterpret_cast<std::uintptr_t>(p1), b2 = reinterpret_cast<std::uintptr_t>(p2);
        const std::uintptr_t len = s.size() * sizeof(T1);
        const bool overlap = b1 < b2 + len && b2 < b1 + len;
        if (!overlap && b1 % 16 == 0 && b2 % 16 == 0) {
          const std::size_t groups = s.size() / (16 / sizeof(T1));
          hipLaunchKernelGGL((detail::for_each_zip2_staged_kernel<T1, T2, Fn>),
                             dim3(detail::gridsize_oneshot(groups, detail::kThreads)), dim3(detail::kThreads), 0,
                             stream(s.rank()), p1, p2, s.size(), fn);
          detail::hip_check(hipGetLastError(), "for_each launch");
          return;
        }
      }
    }
    if constexpr (requires { requires A::stageable; }) {
      using T = std::remove_pointer_t<decltype(a.staged_base())>;
      if constexpr (std::is_trivially_copyable_v<T> && !std::is_const_v<T> && 16 % sizeof(T) == 0) {
        if (reinterpret_cast<std::uintptr_t>(a.staged_base()) % 16 == 0) {
          const std::size_t groups = s.size() / (16 / sizeof(T));
          hipLaunchKernelGGL((detail::for_each_staged_kernel<T, A, Fn>),
                             dim3(detail::gridsize_oneshot(groups, detail::kThreads * detail::kForEachStagedUnroll)),
                             dim3(detail::kThreads), 0, stream(s.rank()), a.staged_base(), a, s.size(), fn);
          detail::hip_check(hipGetLastError(), "for_each launch");
          return;
        }
      }
    }
    hipLaunchKernelGGL((detail::for_each_kernel<decltype(a), Fn>),
                       dim3(detail::gridsize_oneshot(s.size(), detail::kThreads * detail::kForEachUnroll)),
                       dim3(detail::kThreads), 0, stream(s.rank()), a, s.size(), fn);
    detail::hip_check(hipGetLastError(), "for_each launch");
  };
  detail::each_segment(lib::ranges::segments(r), [&](const auto &s) {
    // segments with several accessor shapes (dense tiles: trimmed or not,
    // 32- or 64-bit row division) pick the one that fits, branch-free
    if constexpr (requires { typename std::remove_cvref_t<decltype(s)>::dispatches_accessor; })
      s.visit_accessor([&](auto a) { launch(a, s); });
    else
      launch(detail::accessor_of(s), s);
  });
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter, typename Fn>
void for_each(ExecutionPolicy &&policy, Iter first, Iter last, Fn fn) {
  for_each(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last), fn);
}

// -------------------------------------------------------------- fill / iota
// copy.hpp:147-173: fill_async returns the completion event, fill waits.
template <typename T>
  requires(!std::is_const_v<T>)
event fill_async(device_ptr<T> first, device_ptr<T> last, const T &value) {
  event e;
  if (last - first > 0) {
    detail::fill_segment_async(first.rank(), first.local(), static_cast<std::size_t>(last - first), value);
    e.add(first.rank());
  }
  return e;
}
template <typename T>
  requires(!std::is_const_v<T>)
void fill(device_ptr<T> first, device_ptr<T> last, const T &value) {
  fill_async(first, last, value).wait();
}

template <typename R, typename T>
  requires lib::distributed_contiguous_range<R>
event fill_async(R &&r, const T &value) {
  using V = std::ranges::range_value_t<R>;
  const V v = static_cast<V>(value);
  event e;
  for (auto &&s : lib::ranges::segments(r)) {
    if (!s.size()) continue;
    detail::fill_segment_async(s.rank(), s.data(), s.size(), v);
    e.add(s.rank());
  }
  return e;
}
template <typename R, typename T>
  requires lib::distributed_contiguous_range<R>
void fill(R &&r, const T &value) {
  fill_async(std::forward<R>(r), value).wait();
}
template <lib::distributed_iterator Iter, typename T> event fill_async(Iter first, Iter last, const T &value) {
  return fill_async(std::ranges::subrange(first, last), value);
}
template <lib::distributed_iterator Iter, typename T> void fill(Iter first, Iter last, const T &value) {
  fill_async(first, last, value).wait();
}

// std::iota over a distributed range (test/gtest/shp/algorithms.cpp:11-19),
// one device kernel per segment instead of per-element device_ref writes.
template <typename R, typename T>
  requires lib::distributed_contiguous_range<R>
void iota(R &&r, T start) {
  using V = std::ranges::range_value_t<R>;
  std::size_t off = 0;
  detail::each_segment(lib::ranges::segments(r), [&](const auto &s) {
    const V v0 = static_cast<V>(start + static_cast<T>(off));
    static_assert(detail::abi_type<V>, "shp::iota: element type must be int32/uint32/int64/uint64/float/double");
    detail::check(drhip_iota(static_cast<int>(s.rank()), detail::dtype_code<V>(), s.data(), s.size(), &v0),
                  "drhip_iota");
    off += s.size();
  });
}

// ---------------------------------------------------------------- copy
// copy.hpp:19-145.  copy_async enqueues on the segment streams and returns
// the completion event (the reference's sycl::event); copy waits on it.  A
// pageable host buffer makes the HIP copy itself blocking; pinned host
// memory (drhip_host_alloc) keeps it asynchronous.

// host <-> one device segment (device_ptr), and device_ptr -> device_ptr
template <std::contiguous_iterator Iter, typename T>
  requires(std::is_same_v<std::remove_const_t<std::iter_value_t<Iter>>, T> && !std::is_const_v<T>)
event copy_async(Iter first, Iter last, device_ptr<T> d_first) {
  event e;
  const std::size_t n = static_cast<std::size_t>(last - first);
  if (n) {
    detail::check(drhip_memcpy_h2d(static_cast<int>(d_first.rank()), d_first.local(), std::to_address(first),
                                   n * sizeof(T)),
                  "copy_async h2d");
    e.add(d_first.rank());
  }
  return e;
}
template <std::contiguous_iterator Iter, typename T>
  requires(std::is_same_v<std::remove_const_t<std::iter_value_t<Iter>>, T> && !std::is_const_v<T>)
device_ptr<T> copy(Iter first, Iter last, device_ptr<T> d_first) {
  copy_async(first, last, d_first).wait();
  return d_first + (last - first);
}
template <typename T, std::contiguous_iterator Iter>
  requires(std::is_same_v<std::iter_value_t<Iter>, std::remove_const_t<T>>)
event copy_async(device_ptr<T> first, device_ptr<T> last, Iter d_first) {
  event e;
  const std::size_t n = static_cast<std::size_t>(last - first);
  if (n) {
    detail::check(drhip_memcpy_d2h(static_cast<int>(first.rank()), std::to_address(d_first), first.local(),
                                   n * sizeof(T)),
                  "copy_async d2h");
    e.add(first.rank());
  }
  return e;
}
template <typename T, std::contiguous_iterator Iter>
  requires(std::is_same_v<std::iter_value_t<Iter>, std::remove_const_t<T>>)
Iter copy(device_ptr<T> first, device_ptr<T> last, Iter d_first) {
  copy_async(first, last, d_first).wait();
  return d_first + (last - first);
}
template <typename T, typename U>
  requires(std::is_same_v<std::remove_const_t<T>, U>)
event copy_async(device_ptr<T> first, device_ptr<T> last, device_ptr<U> d_first) {
  event e;
  const std::size_t n = static_cast<std::size_t>(last - first);
  if (n) {
    detail::check(drhip_memcpy_d2d(static_cast<int>(d_first.rank()), d_first.local(), first.local(), n * sizeof(U)),
                  "copy_async d2d");
    e.add(d_first.rank());
  }
  return e;
}
template <typename T, typename U>
  requires(std::is_same_v<std::remove_const_t<T>, U>)
device_ptr<U> copy(device_ptr<T> first, device_ptr<T> last, device_ptr<U> d_first) {
  copy_async(first, last, d_first).wait();
  return d_first + (last - first);
}

// local (host) -> distributed (copy.hpp:71-113): one copy per touched segment
template <std::forward_iterator InputIt, lib::distributed_iterator OutputIt>
  requires(!lib::distributed_iterator<InputIt>)
event copy_async(InputIt first, InputIt last, OutputIt d_first) {
  using V = std::iter_value_t<OutputIt>;
  const std::size_t n = static_cast<std::size_t>(std::distance(first, last));
  event e;
  if constexpr (std::contiguous_iterator<InputIt>) {
    const auto *src = std::to_address(first);
    std::size_t off = 0;
    for (auto &s : d_first.segments_to(d_first + n)) {
      detail::check(drhip_memcpy_h2d(static_cast<int>(s.rank()), s.data(), src + off, s.size() * sizeof(V)),
                    "copy h2d");
      e.add(s.rank());
      off += s.size();
    }
  } else { // any forward iterator: staged through a contiguous host copy
    std::vector<V> stage(first, last);
    e = copy_async(stage.begin(), stage.end(), d_first);
    e.wait();
  }
  return e;
}
template <std::forward_iterator InputIt, lib::distributed_iterator OutputIt>
  requires(!lib::distributed_iterator<InputIt>)
OutputIt copy(InputIt first, InputIt last, OutputIt d_first) {
  const auto n = std::distance(first, last);
  copy_async(first, last, d_first).wait();
  return d_first + n;
}

// distributed -> local (host) (copy.hpp:115-145)
template <lib::distributed_iterator InputIt, std::contiguous_iterator OutputIt>
  requires(!lib::distributed_iterator<OutputIt>)
event copy_async(InputIt first, InputIt last, OutputIt d_first) {
  auto *dst = std::to_address(d_first);
  std::size_t off = 0;
  event e;
  for (auto &s : first.segments_to(last)) {
    detail::check(drhip_memcpy_d2h(static_cast<int>(s.rank()), dst + off, s.data(), s.size() * sizeof(*dst)),
                  "copy d2h");
    e.add(s.rank());
    off += s.size();
  }
  return e;
}
template <lib::distributed_iterator InputIt, std::contiguous_iterator OutputIt>
  requires(!lib::distributed_iterator<OutputIt>)
OutputIt copy(InputIt first, InputIt last, OutputIt d_first) {
  copy_async(first, last, d_first).wait();
  return d_first + (last - first);
}

// distributed -> distributed (peer copies over xGMI where ranks differ)
template <lib::distributed_iterator InputIt, lib::distributed_iterator OutputIt>
event copy_async(InputIt first, InputIt last, OutputIt d_first) {
  const std::size_t n = static_cast<std::size_t>(last - first);
  auto in = first.segments_to(last);
  auto out = d_first.segments_to(d_first + n);
  std::vector<std::size_t> bounds = detail::boundaries(in), bo = detail::boundaries(out);
  bounds.insert(bounds.end(), bo.begin(), bo.end());
  std::sort(bounds.begin(), bounds.end());
  bounds.erase(std::unique(bounds.begin(), bounds.end()), bounds.end());
  auto pi = detail::cut(in, bounds), po = detail::cut(out, bounds);
  event e;
  for (std::size_t k = 0; k < pi.size(); k++) {
    detail::check(drhip_memcpy_d2d(static_cast<int>(po[k].rank()), po[k].data(), pi[k].data(),
                                   pi[k].size() * sizeof(*pi[k].data())),
                  "copy d2d");
    e.add(po[k].rank());
  }
  return e;
}
template <lib::distributed_iterator InputIt, lib::distributed_iterator OutputIt>
OutputIt copy(InputIt first, InputIt last, OutputIt d_first) {
  copy_async(first, last, d_first).wait();
  return d_first + (last - first);
}

template <typename R, typename O>
  requires lib::distributed_range<R>
auto copy(R &&r, O d_first) {
  return shp::copy(std::ranges::begin(r), std::ranges::end(r), d_first);
}

// ----------------------------------------------------------------- reduce
// reduce.hpp:40-88: per-segment partials (the C-ABI kernel for standard
// operators, the template kernel otherwise), then
// init = op(init, partial_k) on the host in segment order (:81-83).
template <typename ExecutionPolicy, typename R, typename T, typename BinaryOp>
  requires lib::distributed_range<R>
T reduce(ExecutionPolicy &&, R &&r, T init, BinaryOp &&binary_op) {
  auto segs = lib::ranges::segments(r);
  using Seg = std::remove_cvref_t<decltype(segs[0])>;
  using V = typename decltype(detail::value_type_of_segment<Seg>())::type;
  constexpr int OP = detail::op_code<BinaryOp>();
  if constexpr (detail::is_device_span<Seg> && detail::abi_type<V> && OP >= 0) {
    using A = detail::abi_acc_t<V>;
    detail::pinned<A> part(segs.size());
    for (std::size_t k = 0; k < segs.size(); k++)
      if (segs[k].size())
        detail::check(drhip_reduce(static_cast<int>(segs[k].rank()), detail::dtype_code<V>(), OP, segs[k].data(),
                                   segs[k].size(), &part[k]),
                      "drhip_reduce");
    for (auto &s : segs) sync(s.rank());
    for (std::size_t k = 0; k < segs.size(); k++)
      if (segs[k].size()) init = static_cast<T>(binary_op(init, static_cast<T>(part[k])));
    return init;
  } else {
    std::vector<detail::maybe<V> *> parts(segs.size(), nullptr);
    std::vector<std::unique_ptr<detail::pinned<detail::maybe<V>>>> held;
    std::vector<int> grids(segs.size(), 0);
    for (std::size_t k = 0; k < segs.size(); k++) {
      if (!segs[k].size()) continue;
      grids[k] = std::min(detail::gridsize_oneshot(segs[k].size(), detail::kThreads * detail::kReduceUnroll),
                          DRHIP_REDUCE_BLOCKS);
      held.emplace_back(std::make_unique<detail::pinned<detail::maybe<V>>>(grids[k]));
      parts[k] = held.back()->data();
      std::remove_cvref_t<BinaryOp> op = binary_op;
      detail::launch_generic_reduce<V>(segs[k], op, grids[k], parts[k]);
    }
    for (auto &s : segs) sync(s.rank());
    for (std::size_t k = 0; k < segs.size(); k++) {
      if (!parts[k]) continue;
      for (int b = 0; b < grids[k]; b++)
        if (parts[k][b].ok) init = static_cast<T>(binary_op(init, parts[k][b].v));
    }
    return init;
  }
}

template <typename ExecutionPolicy, typename R, typename T>
  requires lib::distributed_range<R>
T reduce(ExecutionPolicy &&policy, R &&r, T init) {
  return shp::reduce(std::forward<ExecutionPolicy>(policy), std::forward<R>(r), init, std::plus<>());
}

template <typename ExecutionPolicy, typename R>
  requires lib::distributed_range<R>
auto reduce(ExecutionPolicy &&policy, R &&r) {
  using V = std::ranges::range_value_t<R>;
  return shp::reduce(std::forward<ExecutionPolicy>(policy), std::forward<R>(r), V{}, std::plus<>());
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter>
auto reduce(ExecutionPolicy &&policy, Iter first, Iter last) {
  return shp::reduce(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last));
}
template <typename ExecutionPolicy, lib::distributed_iterator Iter, typename T>
T reduce(ExecutionPolicy &&policy, Iter first, Iter last, T init) {
  return shp::reduce(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last), init);
}
template <typename ExecutionPolicy, lib::distributed_iterator Iter, typename T, typename BinaryOp>
T reduce(ExecutionPolicy &&policy, Iter first, Iter last, T init, BinaryOp &&op) {
  return shp::reduce(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last), init,
                     std::forward<BinaryOp>(op));
}

// ------------------------------------------------------- transform_reduce
// dot_product.cpp:11-18 composition as one call.  plus/multiplies over two
// aligned contiguous ranges of one ABI type is the fused drhip_dot kernel
// (8 B/elem for f32); anything else is reduce(zip | transform).
template <typename ExecutionPolicy, typename R1, typename R2, typename T, typename ROp, typename TOp>
  requires lib::distributed_range<R1> && lib::distributed_range<R2>
T transform_reduce(ExecutionPolicy &&policy, R1 &&r1, R2 &&r2, T init, ROp rop, TOp top) {
  auto z = views::zip(r1, r2);
  auto segs = z.zipped_segments();
  using Z = std::remove_cvref_t<decltype(segs[0])>;
  using S1 = std::remove_cvref_t<decltype(std::get<0>(std::declval<Z>().parts))>;
  using S2 = std::remove_cvref_t<decltype(std::get<1>(std::declval<Z>().parts))>;
  if constexpr (detail::is_device_span<S1> && detail::is_device_span<S2> &&
                detail::op_code<ROp>() == DRHIP_PLUS && detail::op_code<TOp>() == DRHIP_MUL) {
    using V1 = std::remove_cv_t<typename S1::value_type>;
    using V2 = std::remove_cv_t<typename S2::value_type>;
    if constexpr (std::is_same_v<V1, V2> && detail::abi_type<V1>) {
      using A = detail::abi_acc_t<V1>;
      detail::pinned<A> part(segs.size());
      for (std::size_t k = 0; k < segs.size(); k++) {
        auto &[a, b] = segs[k].parts;
        if (a.size())
          detail::check(drhip_dot(static_cast<int>(a.rank()), detail::dtype_code<V1>(), a.data(), b.data(), a.size(),
                                  &part[k]),
                        "drhip_dot");
      }
      for (auto &s : segs) sync(s.rank());
      for (std::size_t k = 0; k < segs.size(); k++)
        if (segs[k].size()) init = static_cast<T>(rop(init, static_cast<T>(part[k])));
      return init;
    }
  }
  auto tv = lib::views::transform(std::move(z), [top](auto &&e) { return top(std::get<0>(e), std::get<1>(e)); });
  return shp::reduce(std::forward<ExecutionPolicy>(policy), tv, init, rop);
}

template <typename ExecutionPolicy, typename R1, typename R2, typename T>
T transform_reduce(ExecutionPolicy &&policy, R1 &&r1, R2 &&r2, T init) {
  return shp::transform_reduce(std::forward<ExecutionPolicy>(policy), std::forward<R1>(r1), std::forward<R2>(r2),
                               init, std::plus<>(), std::multiplies<>());
}

// --------------------------------------------------------- inclusive_scan
// inclusive_scan.hpp:22-148.  The reference scans every zipped piece, scans
// the piece totals on device 0 and then re-reads and rewrites every piece
// k > 0 with x = op(x, carry) (16 B/elem for 4-byte T).  Here:
//   P == 1: one single-pass decoupled-look-back scan (8 B/elem);
//   P  > 1: pieces 0..P-2 reduced by drhip_reduce_tiles (parallel, 4 B/elem;
//           each leaves its piece's tile prefixes), the totals in pinned
//           memory every device reads, then every piece's scan -- the tile
//           scan for pieces 0..P-2, the single-pass gathered scan for the
//           last -- folding init and the totals before it on the device
//           (fp64 for fp32): 12 B/elem, no host round trip between the
//           phases.  When two of pieces 0..P-2 share a segment (misaligned
//           zips), the totals are folded on the host and every piece runs
//           the single-pass scan with its carry.
// init applies to piece 0 only (:77-83).  On the C-ABI path (standard,
// commutative operators) the carry enters as op(carry, x), value-identical
// to the reference's op(x, carry); the template path (scan.hpp) keeps the
// reference's operand order for any operator.
namespace detail {

template <typename R, typename O, typename BinaryOp, typename U>
void inclusive_scan_impl(R &&r, O &&o, BinaryOp &&op, std::optional<U> init, bool exclusive) {
  auto z = views::zip(r, o);
  auto pieces = z.zipped_segments();
  using Z = std::remove_cvref_t<decltype(pieces[0])>;
  using SI = std::remove_cvref_t<decltype(std::get<0>(std::declval<Z>().parts))>;
  using SO = std::remove_cvref_t<decltype(std::get<1>(std::declval<Z>().parts))>;
  using TI = typename decltype(detail::value_type_of_segment<SI>())::type;
  using T = std::remove_cv_t<std::ranges::range_value_t<O>>;
  constexpr int OP = detail::op_code<BinaryOp>();
  const std::size_t P = pieces.size();
  if (P == 0) return;

  if constexpr (detail::is_device_span<SI> && detail::is_device_span<SO> && std::is_same_v<TI, T> &&
                detail::abi_type<T> && OP >= 0) {
    if (!exclusive && P > 1) {
      // pieces 0..P-2 on distinct segments: drhip_reduce_tiles leaves each
      // piece's tile prefixes, so its scan is drhip_inclusive_scan_tiles;
      // the piece totals (and init) go to pinned memory that every device
      // reads, and each scan kernel folds the totals before its piece itself
      // (carry = init op t_0 op ... op t_{k-1}): no host round trip between
      // the two phases, only event waits across the segment streams.
      std::vector<std::size_t> rk(P);
      for (std::size_t k = 0; k < P; k++) rk[k] = std::get<0>(pieces[k].parts).rank();
      bool distinct = true;
      for (std::size_t k = 0; k + 1 < P && distinct; k++)
        for (std::size_t j = 0; j < k; j++) distinct = distinct && rk[j] != rk[k];
      if (distinct) {
        using A = detail::abi_acc_t<T>;
        const std::size_t hi = init ? 1 : 0, w = (P - 1) + hi;
        // one spare slot: the last piece folds ALL w values (rank = w < w + 1)
        detail::pinned<A> parts(w + 1);
        if (init) parts[0] = static_cast<A>(*init);
        parts[w] = A{};
        std::vector<hipEvent_t> ev(P - 1);
        for (std::size_t k = 0; k + 1 < P; k++) {
          auto &[in, out] = pieces[k].parts;
          detail::check(drhip_reduce_tiles(static_cast<int>(rk[k]), detail::dtype_code<T>(), OP, in.data(),
                                           in.size(), &parts[k + hi]),
                        "drhip_reduce_tiles");
          detail::hip_check(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "hipEventCreate");
          detail::hip_check(hipEventRecord(ev[k], stream(rk[k])), "hipEventRecord");
        }
        for (std::size_t k = 0; k < P; k++)
          for (std::size_t j = 0; j + 1 < P; j++)
            if (rk[j] != rk[k]) detail::hip_check(hipStreamWaitEvent(stream(rk[k]), ev[j], 0), "hipStreamWaitEvent");
        for (std::size_t k = 0; k < P; k++) {
          auto &[in, out] = pieces[k].parts;
          if (k + 1 < P)
            detail::check(drhip_inclusive_scan_tiles(static_cast<int>(rk[k]), detail::dtype_code<T>(), OP,
                                                     in.data(), out.data(), in.size(), nullptr, &parts[0],
                                                     static_cast<int>(w + 1), static_cast<int>(k + hi), nullptr),
                          "drhip_inclusive_scan_tiles");
          else
            detail::check(drhip_inclusive_scan_gathered(static_cast<int>(rk[k]), detail::dtype_code<T>(), OP,
                                                        in.data(), out.data(), in.size(), &parts[0],
                                                        static_cast<int>(w + 1), static_cast<int>(w), nullptr),
                          "drhip_inclusive_scan_gathered");
        }
        for (auto &p : pieces) sync(p.rank());
        for (auto &e : ev) (void)hipEventDestroy(e);
        return;
      }
    }
    if (!exclusive) {
      using A = detail::abi_acc_t<T>;
      std::vector<A> carry(P);
      std::vector<bool> has_carry(P, false);
      if (P > 1) {
        detail::pinned<A> tot(P);
        for (std::size_t k = 0; k + 1 < P; k++) {
          auto &[in, out] = pieces[k].parts;
          detail::check(drhip_reduce(static_cast<int>(in.rank()), detail::dtype_code<T>(), OP, in.data(), in.size(),
                                     &tot[k]),
                        "drhip_reduce");
        }
        for (std::size_t k = 0; k + 1 < P; k++) sync(std::get<0>(pieces[k].parts).rank());
        A run{};
        bool ok = false;
        if (init) {
          run = static_cast<A>(*init);
          ok = true;
        }
        for (std::size_t k = 1; k < P; k++) {
          run = ok ? static_cast<A>(op(run, tot[k - 1])) : tot[k - 1];
          ok = true;
          carry[k] = run;
          has_carry[k] = true;
        }
      }
      for (std::size_t k = 0; k < P; k++) {
        auto &[in, out] = pieces[k].parts;
        T iv = init ? static_cast<T>(*init) : T{};
        detail::check(drhip_inclusive_scan(static_cast<int>(in.rank()), detail::dtype_code<T>(), OP, in.data(),
                                           out.data(), in.size(), (k == 0 && init) ? &iv : nullptr,
                                           has_carry[k] ? &carry[k] : nullptr, nullptr, nullptr),
                      "drhip_inclusive_scan");
      }
      for (auto &p : pieces) sync(p.rank());
      return;
    }
  }
  // generic path (any op / view / exclusive): single-pass look-back scans
  // (scan.hpp).  P > 1: the totals of pieces 0..P-2 first (the same kernel
  // in fold-only mode, order kept, 4 B/elem, all pieces concurrently), the
  // running fold of the totals on the host, then every piece's scan with
  // its carry (8 B/elem, concurrently).  Inclusive: S_{k-1} on the right of
  // piece k (inclusive_scan.hpp:132-134); exclusive (std semantics): the
  // fold of init and everything before the piece on the left.
  std::remove_cvref_t<BinaryOp> f = op;
  pinned<T> tot(P);
  pinned<unsigned> err(1);
  err[0] = 0;
  const bool has_init = init.has_value();
  const T iv = has_init ? static_cast<T>(*init) : T{};
  std::vector<T> lc(P, iv), rc(P, iv);
  std::vector<char> hl(P, 0), hr(P, 0);
  hl[0] = has_init;
  auto wait = [&](std::size_t upto) {
    std::vector<std::size_t> ranks;
    for (std::size_t k = 0; k < upto; k++) ranks.push_back(std::get<0>(pieces[k].parts).rank());
    std::sort(ranks.begin(), ranks.end());
    ranks.erase(std::unique(ranks.begin(), ranks.end()), ranks.end());
    for (auto rk : ranks) sync(rk);
    if (err[0] & 2u) throw std::runtime_error("shp: look-back scan: a tile claim past the grid (counter not reset)");
    if (err[0]) throw std::runtime_error("shp: look-back scan: a bounded in-kernel spin timed out");
  };
  if (P > 1) {
    for (std::size_t k = 0; k + 1 < P; k++) {
      auto &[in, out] = pieces[k].parts;
      // inclusive: p_0 includes init (the last element of piece 0's scan)
      lb_scan_launch<T>(in, out, f, !exclusive && k == 0 && has_init, iv, false, iv, false, true, &tot[k], err.data());
    }
    wait(P - 1);
    if (!exclusive) {
      T run = tot[0];
      for (std::size_t k = 1; k < P; k++) {
        rc[k] = run;
        hr[k] = 1;
        if (k + 1 < P) run = static_cast<T>(op(run, tot[k]));
      }
    } else {
      T run = iv;
      for (std::size_t k = 1; k < P; k++) {
        run = static_cast<T>(op(run, tot[k - 1]));
        lc[k] = run;
        hl[k] = 1;
      }
    }
  }
  for (std::size_t k = 0; k < P; k++) {
    auto &[in, out] = pieces[k].parts;
    lb_scan_launch<T>(in, out, f, hl[k] != 0, lc[k], hr[k] != 0, rc[k], exclusive, false, nullptr, err.data());
  }
  wait(P);
}

} // namespace detail

template <typename ExecutionPolicy, typename R, typename O, typename BinaryOp, typename T>
  requires lib::distributed_range<R> && lib::distributed_range<O>
void inclusive_scan(ExecutionPolicy &&, R &&r, O &&o, BinaryOp &&op, T init) {
  detail::inclusive_scan_impl(r, o, op, std::optional<T>(init), false);
}
template <typename ExecutionPolicy, typename R, typename O, typename BinaryOp>
  requires lib::distributed_range<R> && lib::distributed_range<O>
void inclusive_scan(ExecutionPolicy &&, R &&r, O &&o, BinaryOp &&op) {
  detail::inclusive_scan_impl(r, o, op, std::optional<std::ranges::range_value_t<R>>(), false);
}
template <typename ExecutionPolicy, typename R, typename O>
  requires lib::distributed_range<R> && lib::distributed_range<O>
void inclusive_scan(ExecutionPolicy &&policy, R &&r, O &&o) {
  shp::inclusive_scan(std::forward<ExecutionPolicy>(policy), r, o, std::plus<>());
}

// inclusive_scan.hpp:150-218 iterator forms: return d_first + (last - first)
template <typename ExecutionPolicy, lib::distributed_iterator Iter, lib::distributed_iterator OutputIter,
          typename BinaryOp, typename T>
OutputIter inclusive_scan(ExecutionPolicy &&policy, Iter first, Iter last, OutputIter d_first, BinaryOp &&op,
                          T init) {
  auto d_last = d_first + (last - first);
  shp::inclusive_scan(policy, std::ranges::subrange(first, last), std::ranges::subrange(d_first, d_last), op, init);
  return d_last;
}
template <typename ExecutionPolicy, lib::distributed_iterator Iter, lib::distributed_iterator OutputIter,
          typename BinaryOp>
OutputIter inclusive_scan(ExecutionPolicy &&policy, Iter first, Iter last, OutputIter d_first, BinaryOp &&op) {
  auto d_last = d_first + (last - first);
  shp::inclusive_scan(policy, std::ranges::subrange(first, last), std::ranges::subrange(d_first, d_last), op);
  return d_last;
}
template <typename ExecutionPolicy, lib::distributed_iterator Iter, lib::distributed_iterator OutputIter>
OutputIter inclusive_scan(ExecutionPolicy &&policy, Iter first, Iter last, OutputIter d_first) {
  return shp::inclusive_scan(policy, first, last, d_first, std::plus<>());
}

// exclusive_scan (not in the reference snapshot; std:: semantics)
template <typename ExecutionPolicy, typename R, typename O, typename T, typename BinaryOp>
  requires lib::distributed_range<R> && lib::distributed_range<O>
void exclusive_scan(ExecutionPolicy &&, R &&r, O &&o, T init, BinaryOp &&op) {
  detail::inclusive_scan_impl(r, o, op, std::optional<T>(init), true);
}
template <typename ExecutionPolicy, typename R, typename O, typename T>
  requires lib::distributed_range<R> && lib::distributed_range<O>
void exclusive_scan(ExecutionPolicy &&policy, R &&r, O &&o, T init) {
  shp::exclusive_scan(policy, r, o, init, std::plus<>());
}

} // namespace shp
