// stencil.hip -- halo'd 1-D and 2-D stencil steps for gfx950.
//
// The reference's stencil is an mhp (CPU/MPI) construct: a
// distributed_vector with halo_bounds (mhp/containers/distributed_vector.hpp:
// 190-207), span_halo exchange (details/halo.hpp:336-387) and
// mhp::transform of a pointer-offset lambda (mhp/algorithms/
// cpu_algorithms.hpp:147-161, examples/mhp/stencil-1d.cpp:16-19).  On
// MI355X the segment lives in HBM with its halo cells in the same buffer
// ([r halo | owned | r halo]); this kernel is the per-segment transform,
// the exchange is a peer copy / RCCL send-recv of r cells per side.
// HBM bytes per cell per step: 4 read + 4 written (f32/i32); the radius
// neighbours are L1/L2 hits.
#include "common.hpp"

namespace drhip {

constexpr int kStThreads = 256;

template <typename T, int R>
__global__ __launch_bounds__(kStThreads) void stencil1d_kernel(const T *__restrict__ in,
                                                              T *__restrict__ out, size_t lo,
                                                              size_t hi) {
  using C = typename ctype_of<T>::type;
  // LDS tile of kStThreads*4 outputs + 2R halo.
  constexpr int W = kStThreads * 4;
  __shared__ C tile[W + 2 * R];
  const size_t stride = (size_t)gridDim.x * W;
  for (size_t t0 = lo + (size_t)blockIdx.x * W; t0 < hi; t0 += stride) {
    // in index of output i is (R + i); tile[k] = in[t0 + k] covers R+i-R .. R+i+R
    for (int k = threadIdx.x; k < W + 2 * R; k += kStThreads) {
      size_t g = t0 + k;
      tile[k] = g < hi + 2 * R ? (C)in[g] : C(0);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      int li = q * kStThreads + threadIdx.x;
      size_t i = t0 + li;
      if (i < hi) {
        C s = C(0);
#pragma unroll
        for (int d = 0; d <= 2 * R; d++) s += tile[li + d];
        out[R + i] = (T)s;
      }
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(kStThreads) void stencil1d_generic(const T *__restrict__ in,
                                                               T *__restrict__ out, int r, size_t lo,
                                                               size_t hi) {
  using C = typename ctype_of<T>::type;
  const size_t stride = (size_t)gridDim.x * kStThreads;
  for (size_t i = lo + (size_t)blockIdx.x * kStThreads + threadIdx.x; i < hi; i += stride) {
    C s = C(0);
    for (int d = -r; d <= r; d++) s += (C)in[r + i + d];
    out[r + i] = (T)s;
  }
}

template <typename T>
__global__ __launch_bounds__(kStThreads) void stencil2d_kernel(const T *__restrict__ in,
                                                              T *__restrict__ out, size_t nx,
                                                              size_t rlo, size_t rhi) {
  using C = typename ctype_of<T>::type;
  // buffer row (1 + r) holds owned row r; columns 1..nx-2 are interior.
  const size_t inner = nx - 2;
  const size_t total = (rhi - rlo) * inner;
  const size_t stride = (size_t)gridDim.x * kStThreads;
  for (size_t k = (size_t)blockIdx.x * kStThreads + threadIdx.x; k < total; k += stride) {
    size_t r = rlo + k / inner, x = 1 + k % inner;
    size_t c = (1 + r) * nx + x;
    C s = (C)in[c] + (C)in[c - 1] + (C)in[c + 1] + (C)in[c - nx] + (C)in[c + nx];
    out[c] = (T)s;
  }
}

// Vectorised 1-D stencil (radius R <= 16 B / sizeof(T)): lane k owns the
// 16-byte vector of buffer elements [kV, kV+V); its neighbours' vectors come
// from lanes k-1 / k+1 by DPP wave shifts, so every input byte is loaded once
// per wave (the wave's two edge lanes reload one neighbour vector).  Outputs
// are buffer indices [lo_b, hi_b); the window is summed left to right like
// the reference's stencil_op (examples/mhp/stencil-1d.cpp:16-19), so fp32
// results are bit-identical to the oracle.  in/out must be 16-byte aligned.
template <typename T, int R>
__global__ __launch_bounds__(kStThreads) void stencil1d_vec(const T *__restrict__ in, T *__restrict__ out,
                                                           size_t nbuf, size_t lo_b, size_t hi_b) {
  using C = typename ctype_of<T>::type;
  constexpr int V = Vec16<T>::N;
  static_assert(R <= V, "the neighbour vectors cover the radius");
  const int lane = threadIdx.x & (kWave - 1);
  const size_t nfull = nbuf / V;
  const size_t k0 = lo_b / V, k1 = (hi_b + V - 1) / V;
  const Vec16<T> *iv = reinterpret_cast<const Vec16<T> *>(in);
  Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out);
  auto load = [&](size_t kk, Vec16<T> &r, bool nt) {
    if (kk < nfull) {
      r = nt ? load_nt(iv + kk) : iv[kk];
    } else {
#pragma unroll
      for (int j = 0; j < V; j++) {
        const size_t b = kk * V + j;
        r.v[j] = b < nbuf ? in[b] : T(0);
      }
    }
  };
  // wave-uniform loop: every lane takes part in the DPP moves
  const size_t wave = ((size_t)blockIdx.x * kStThreads + threadIdx.x) / kWave;
  const size_t nwaves = (size_t)gridDim.x * (kStThreads / kWave);
  for (size_t kb = k0 + wave * kWave; kb < k1; kb += nwaves * kWave) {
    const size_t k = kb + lane;
    Vec16<T> cur, prv, nxt;
    load(k, cur, true);
#pragma unroll
    for (int j = 0; j < V; j++) {
      prv.v[j] = wave_shift_up1(cur.v[j], T(0));
      nxt.v[j] = wave_shift_down1(cur.v[j], T(0));
    }
    if (lane == 0 && k > 0) load(k - 1, prv, false);
    if (lane == kWave - 1) load(k + 1, nxt, false);
    if (k < k1) {
      C w[3 * V];
#pragma unroll
      for (int j = 0; j < V; j++) {
        w[j] = (C)prv.v[j];
        w[V + j] = (C)cur.v[j];
        w[2 * V + j] = (C)nxt.v[j];
      }
      Vec16<T> o;
      bool whole = true;
#pragma unroll
      for (int j = 0; j < V; j++) {
        C s = C(0);
#pragma unroll
        for (int d = -R; d <= R; d++) s += w[V + j + d];
        o.v[j] = (T)s;
        const size_t b = k * V + j;
        whole &= b >= lo_b && b < hi_b;
      }
      if (whole) {
        store_nt(ov + k, o);
      } else {
#pragma unroll
        for (int j = 0; j < V; j++) {
          const size_t b = k * V + j;
          if (b >= lo_b && b < hi_b) out[b] = o.v[j];
        }
      }
    }
  }
}

// Vectorised 5-point 2-D stencil on a row block ((rows+2) x nx buffer, nx a
// multiple of the vector width, 16-byte aligned): lane k owns buffer vector
// k (elements [kV, kV+V) of the flattened buffer); north/south are the
// vectors nx/V away, west/east come from lanes k-1 / k+1 by DPP wave shifts
// (a row's first and last vectors never need the neighbour across the row
// edge: columns 0 and nx-1 are not interior).  Same summation order as the
// oracle: c + w + e + n + s.
template <typename T>
__global__ __launch_bounds__(kStThreads) void stencil2d_vec(const T *__restrict__ in, T *__restrict__ out,
                                                           size_t nx, size_t rlo, size_t rhi) {
  using C = typename ctype_of<T>::type;
  constexpr int V = Vec16<T>::N;
  const int lane = threadIdx.x & (kWave - 1);
  const size_t vpr = nx / V;                      // vectors per row
  const size_t k0 = (1 + rlo) * vpr, k1 = (1 + rhi) * vpr;
  const Vec16<T> *iv = reinterpret_cast<const Vec16<T> *>(in);
  Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out);
  const size_t wave = ((size_t)blockIdx.x * kStThreads + threadIdx.x) / kWave;
  const size_t nwaves = (size_t)gridDim.x * (kStThreads / kWave);
  for (size_t kb = k0 + wave * kWave; kb < k1; kb += nwaves * kWave) {
    const size_t k = kb + lane;
    const bool act = k < k1;
    Vec16<T> c{}, nn{}, ss{};
    if (act) {
      c = iv[k];
      nn = iv[k - vpr];
      ss = iv[k + vpr];
    }
    Vec16<T> w, e;
#pragma unroll
    for (int j = 0; j < V; j++) {
      w.v[j] = wave_shift_up1(c.v[j], T(0));
      e.v[j] = wave_shift_down1(c.v[j], T(0));
    }
    if (act && lane == 0) w = iv[k - 1];
    if (act && lane == kWave - 1) e = iv[k + 1];
    if (act) {
      const size_t q = k % vpr; // vector index inside the row
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < V; j++) {
        const C west = j == 0 ? (C)w.v[V - 1] : (C)c.v[j - 1];
        const C east = j == V - 1 ? (C)e.v[0] : (C)c.v[j + 1];
        o.v[j] = (T)((C)c.v[j] + west + east + (C)nn.v[j] + (C)ss.v[j]);
      }
      if (q != 0 && q != vpr - 1) {
        ov[k] = o;
      } else {
        // row edge vector: column 0 / nx-1 are not interior
        T *dst = out + k * V;
#pragma unroll
        for (int j = 0; j < V; j++) {
          const size_t col = q * V + j;
          if (col >= 1 && col + 1 < nx) dst[j] = o.v[j];
        }
      }
    }
  }
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_stencil1d(int seg, int dtype, const void *in_buf, void *out_buf, size_t n_owned,
                               int radius, size_t lo, size_t hi) {
  DRHIP_GET_SEG(s, seg);
  if (radius < 0 || hi > n_owned || lo > hi) return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil1d: bounds");
  if (lo == hi) return DRHIP_OK;
  if (!in_buf || !out_buf) return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil1d: null");
  auto go = [&](auto tv) -> int {
    using T = decltype(tv);
    DRHIP_CHECK_HIP(hipSetDevice(s->device));
    size_t work = hi - lo;
    constexpr int V = Vec16<T>::N;
    const bool aligned = ((uintptr_t)in_buf % 16 == 0) && ((uintptr_t)out_buf % 16 == 0);
    if (aligned && radius >= 1 && radius <= V && radius <= 4) {
      const size_t nvec = (work + V - 1) / V + 1;
      unsigned grid = (unsigned)std::min<size_t>((nvec + kStThreads - 1) / kStThreads, (size_t)s->num_cus * 8);
      const size_t nbuf = n_owned + 2 * (size_t)radius, lo_b = radius + lo, hi_b = radius + hi;
#define DRHIP_ST(RR)                                                                                 \
  hipLaunchKernelGGL((stencil1d_vec<T, RR>), dim3(grid), dim3(kStThreads), 0, s->stream, (const T *)in_buf, \
                     (T *)out_buf, nbuf, lo_b, hi_b)
      if (radius == 1) DRHIP_ST(1);
      else if (radius == 2) DRHIP_ST(2);
      else if constexpr (V >= 4) {
        if (radius == 3) DRHIP_ST(3);
        else DRHIP_ST(4);
      }
#undef DRHIP_ST
    } else if (radius == 1) {
      unsigned grid = (unsigned)std::min<size_t>((work + kStThreads * 4 - 1) / (kStThreads * 4),
                                                 (size_t)s->num_cus * 8);
      hipLaunchKernelGGL((stencil1d_kernel<T, 1>), dim3(grid), dim3(kStThreads), 0, s->stream,
                         (const T *)in_buf, (T *)out_buf, lo, hi);
    } else {
      unsigned grid = (unsigned)std::min<size_t>((work + kStThreads - 1) / kStThreads, (size_t)s->num_cus * 8);
      hipLaunchKernelGGL((stencil1d_generic<T>), dim3(grid), dim3(kStThreads), 0, s->stream,
                         (const T *)in_buf, (T *)out_buf, radius, lo, hi);
    }
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  };
  if (dtype == DRHIP_F32) return go(float{});
  if (dtype == DRHIP_I32) return go(int32_t{});
  if (dtype == DRHIP_F64) return go(double{});
  if (dtype == DRHIP_I64) return go(int64_t{});
  return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil1d: dtype");
}

extern "C" int drhip_stencil2d(int seg, int dtype, const void *in_buf, void *out_buf, size_t nx, size_t rows,
                               size_t rlo, size_t rhi) {
  DRHIP_GET_SEG(s, seg);
  if (rhi > rows || rlo > rhi || nx < 3) return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil2d: bounds");
  if (rlo == rhi) return DRHIP_OK;
  if (!in_buf || !out_buf) return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil2d: null");
  auto go = [&](auto tv) -> int {
    using T = decltype(tv);
    DRHIP_CHECK_HIP(hipSetDevice(s->device));
    size_t work = (rhi - rlo) * (nx - 2);
    constexpr int V = Vec16<T>::N;
    const bool vec = nx % V == 0 && nx >= 2 * V && ((uintptr_t)in_buf % 16 == 0) && ((uintptr_t)out_buf % 16 == 0);
    if (vec) {
      const size_t nvec = (rhi - rlo) * (nx / V);
      unsigned grid = (unsigned)std::min<size_t>((nvec + kStThreads - 1) / kStThreads, (size_t)s->num_cus * 8);
      hipLaunchKernelGGL((stencil2d_vec<T>), dim3(grid), dim3(kStThreads), 0, s->stream, (const T *)in_buf,
                         (T *)out_buf, nx, rlo, rhi);
    } else {
      unsigned grid = (unsigned)std::min<size_t>((work + kStThreads - 1) / kStThreads, (size_t)s->num_cus * 8);
      hipLaunchKernelGGL((stencil2d_kernel<T>), dim3(grid), dim3(kStThreads), 0, s->stream, (const T *)in_buf,
                         (T *)out_buf, nx, rlo, rhi);
    }
    DRHIP_CHECK_LAUNCH();
    return DRHIP_OK;
  };
  if (dtype == DRHIP_F32) return go(float{});
  if (dtype == DRHIP_I32) return go(int32_t{});
  return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil2d: dtype F32 or I32");
}
