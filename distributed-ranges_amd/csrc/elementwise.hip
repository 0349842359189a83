// elementwise.hip -- fill / iota / transform kernels for gfx950.
//
// Fixed-function forms of the reference's per-segment SYCL kernels:
//   fill_async        shp/copy.hpp:147-168 (queue.fill), and the zero fill
//                     of distributed_vector construction
//                     (shp/distributed_vector.hpp:153)
//   iota              std::iota over a distributed_vector
//                     (test/gtest/shp/algorithms.cpp:11-19)
//   for_each          shp/algorithms/for_each.hpp:38-39 (parallel_for,
//                     one work-item per element) -- fixed ops only; user
//                     lambdas take the header-only template path.
// All are grid-stride loops launched one-shot (one 16-byte vector per
// thread; tools/copy_sweep.hip: a one-shot grid with nontemporal load +
// store streams 6.6 TB/s read+write, ahead of every persistent shape),
// 16-byte vector loads/stores when the pointers are 16-byte aligned,
// HBM-bound (fill 4 B/elem written, transform 8 B/elem).
#include "common.hpp"

namespace drhip {

constexpr int kEwThreads = 256;
constexpr size_t kEwMaxBlocks = size_t(1) << 22; // grid-stride beyond 2^30 vectors

template <typename T> struct FillF {
  T v;
  __device__ T operator()(T, size_t) const { return v; }
};
template <typename T> struct IotaF {
  T start;
  __device__ T operator()(T, size_t i) const {
    using C = typename ctype_of<T>::type;
    return (T)((C)start + (C)i);
  }
};
template <typename T, int OP> struct ScalarF {
  T s;
  __device__ T operator()(T x, size_t) const {
    using C = typename compute_of<OP, T>::type;
    return (T)Op<OP, C>::apply((C)x, (C)s);
  }
};
template <typename T> struct NegF {
  __device__ T operator()(T x, size_t) const {
    using C = typename ctype_of<T>::type;
    if constexpr (std::is_floating_point_v<T>) return -x;
    else return (T)(C(0) - (C)x);
  }
};

// out[i] = f(in[i], i).  READ=false: `in` is not read (fill / iota).
template <typename T, typename F, bool READ, bool VEC>
__global__ __launch_bounds__(kEwThreads) void unary_kernel(const T *in, T *out, size_t n, F f) {
  const size_t stride = (size_t)gridDim.x * kEwThreads;
  size_t i = (size_t)blockIdx.x * kEwThreads + threadIdx.x;
  if (VEC) {
    constexpr int V = Vec16<T>::N;
    const size_t nv = n / V;
    const Vec16<T> *iv = reinterpret_cast<const Vec16<T> *>(in);
    Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out);
    for (size_t k = i; k < nv; k += stride) {
      Vec16<T> r;
      if (READ) r = load_nt(iv + k);
#pragma unroll
      for (int j = 0; j < V; j++) r.v[j] = f(READ ? r.v[j] : T(0), k * V + j);
      store_nt(ov + k, r);
    }
    for (size_t k = nv * V + i; k < n; k += stride) out[k] = f(READ ? in[k] : T(0), k);
  } else {
    for (size_t k = i; k < n; k += stride) out[k] = f(READ ? in[k] : T(0), k);
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kEwThreads) void binary_kernel(const T *a, const T *b, T *out, size_t n) {
  using C = typename compute_of<OP, T>::type;
  const size_t stride = (size_t)gridDim.x * kEwThreads;
  for (size_t k = (size_t)blockIdx.x * kEwThreads + threadIdx.x; k < n; k += stride)
    out[k] = (T)Op<OP, C>::apply((C)a[k], (C)b[k]);
}

template <typename T, int OP>
__global__ __launch_bounds__(kEwThreads) void binary_kernel_vec(const T *a, const T *b, T *out,
                                                                size_t n) {
  using C = typename compute_of<OP, T>::type;
  constexpr int V = Vec16<T>::N;
  const size_t stride = (size_t)gridDim.x * kEwThreads;
  const size_t nv = n / V;
  const Vec16<T> *av = reinterpret_cast<const Vec16<T> *>(a);
  const Vec16<T> *bv = reinterpret_cast<const Vec16<T> *>(b);
  Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out);
  size_t i = (size_t)blockIdx.x * kEwThreads + threadIdx.x;
  for (size_t k = i; k < nv; k += stride) {
    Vec16<T> x = load_nt(av + k), y = load_nt(bv + k), r;
#pragma unroll
    for (int j = 0; j < V; j++) r.v[j] = (T)Op<OP, C>::apply((C)x.v[j], (C)y.v[j]);
    store_nt(ov + k, r);
  }
  for (size_t k = nv * V + i; k < n; k += stride) out[k] = (T)Op<OP, C>::apply((C)a[k], (C)b[k]);
}

static unsigned ew_grid(const Segment *s, size_t work) {
  size_t g = (work + kEwThreads - 1) / kEwThreads;
  return (unsigned)std::max<size_t>(1, std::min(g, kEwMaxBlocks));
}

static bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

template <typename T, bool READ, typename F>
static int launch_unary(Segment *s, const T *in, T *out, size_t n, F f) {
  if (n == 0) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  bool vec = aligned16(out) && (!READ || aligned16(in));
  unsigned grid = ew_grid(s, vec ? n / Vec16<T>::N + 1 : n);
  if (vec)
    hipLaunchKernelGGL((unary_kernel<T, F, READ, true>), dim3(grid), dim3(kEwThreads), 0, s->stream, in,
                       out, n, f);
  else
    hipLaunchKernelGGL((unary_kernel<T, F, READ, false>), dim3(grid), dim3(kEwThreads), 0, s->stream, in,
                       out, n, f);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_fill(int seg, void *dst, size_t n, const void *value_host, size_t elem_size) {
  DRHIP_GET_SEG(s, seg);
  if ((!dst && n) || !value_host) return set_error(DRHIP_ERR_BAD_ARG, "drhip_fill: null pointer");
  switch (elem_size) {
  case 1: {
    DRHIP_CHECK_HIP(hipSetDevice(s->device));
    DRHIP_CHECK_HIP(hipMemsetAsync(dst, *(const unsigned char *)value_host, n, s->stream));
    return DRHIP_OK;
  }
  case 2: {
    uint16_t v;
    memcpy(&v, value_host, 2);
    return launch_unary<uint16_t, false>(s, nullptr, (uint16_t *)dst, n, FillF<uint16_t>{v});
  }
  case 4: {
    uint32_t v;
    memcpy(&v, value_host, 4);
    return launch_unary<uint32_t, false>(s, nullptr, (uint32_t *)dst, n, FillF<uint32_t>{v});
  }
  case 8: {
    uint64_t v;
    memcpy(&v, value_host, 8);
    return launch_unary<uint64_t, false>(s, nullptr, (uint64_t *)dst, n, FillF<uint64_t>{v});
  }
  default: return set_error(DRHIP_ERR_BAD_ARG, "drhip_fill: element size must be 1, 2, 4 or 8");
  }
}

extern "C" int drhip_iota(int seg, int dtype, void *dst, size_t n, const void *start_host) {
  DRHIP_GET_SEG(s, seg);
  if ((!dst && n) || !start_host) return set_error(DRHIP_ERR_BAD_ARG, "drhip_iota: null pointer");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    T start;
    memcpy(&start, start_host, sizeof(T));
    return launch_unary<T, false>(s, nullptr, (T *)dst, n, IotaF<T>{start});
  });
}

extern "C" int drhip_transform_scalar(int seg, int dtype, int op, const void *in, void *out, size_t n,
                                      const void *scalar_host) {
  DRHIP_GET_SEG(s, seg);
  if (((!in || !out) && n) || !scalar_host) return set_error(DRHIP_ERR_BAD_ARG, "drhip_transform_scalar: null");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    T sc;
    memcpy(&sc, scalar_host, sizeof(T));
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      return launch_unary<T, true>(s, (const T *)in, (T *)out, n, ScalarF<T, OP>{sc});
    });
  });
}

extern "C" int drhip_negate(int seg, int dtype, void *x, size_t n) {
  DRHIP_GET_SEG(s, seg);
  if (!x && n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_negate: null");
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return launch_unary<T, true>(s, (const T *)x, (T *)x, n, NegF<T>{});
  });
}

extern "C" int drhip_transform_binary(int seg, int dtype, int op, const void *a, const void *b, void *out,
                                      size_t n) {
  DRHIP_GET_SEG(s, seg);
  if ((!a || !b || !out) && n) return set_error(DRHIP_ERR_BAD_ARG, "drhip_transform_binary: null");
  if (n == 0) return DRHIP_OK;
  return dispatch_dtype(dtype, [&](auto tv) -> int {
    using T = decltype(tv);
    return dispatch_op(op, [&](auto ov) -> int {
      constexpr int OP = decltype(ov)::value;
      DRHIP_CHECK_HIP(hipSetDevice(s->device));
      bool vec = aligned16(a) && aligned16(b) && aligned16(out);
      unsigned grid = ew_grid(s, vec ? n / Vec16<T>::N + 1 : n);
      if (vec)
        hipLaunchKernelGGL((binary_kernel_vec<T, OP>), dim3(grid), dim3(kEwThreads), 0, s->stream,
                           (const T *)a, (const T *)b, (T *)out, n);
      else
        hipLaunchKernelGGL((binary_kernel<T, OP>), dim3(grid), dim3(kEwThreads), 0, s->stream,
                           (const T *)a, (const T *)b, (T *)out, n);
      DRHIP_CHECK_LAUNCH();
      return DRHIP_OK;
    });
  });
}
