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

#include <cstdlib>
#include <type_traits>

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
        C s = tile[li];
#pragma unroll
        for (int d = 1; d <= 2 * R; d++) s += tile[li + d];
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
    C s = (C)in[i];
    for (int d = -r + 1; d <= r; d++) s += (C)in[r + i + d];
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
// 16-byte vector of buffer elements [kV, kV+V); its neighbours' elements
// come from lanes k-1 / k+1 by DPP wave shifts, and the wave's two edge
// lanes load just the R elements across the wave edge (scalar loads that hit
// the lines the neighbouring waves fetch).  One vector per thread, one-shot
// grid, cached loads and stores: tools/stencil_sweep.hip measured this shape
// at 6.17 TB/s against 5.10 TB/s for nontemporal loads with whole-vector
// edge reloads.  Outputs are buffer indices [lo_b, hi_b); the window is
// summed left to right from its first term like the reference's stencil_op
// (examples/mhp/stencil-1d.cpp:16-19), so results are bit-identical to the
// oracle.  in/out must be 16-byte aligned.
template <typename T, int R, int NT = 0>
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
  // wave-uniform loop: every lane takes part in the DPP moves
  const size_t wave = ((size_t)blockIdx.x * kStThreads + threadIdx.x) / kWave;
  const size_t nwaves = (size_t)gridDim.x * (kStThreads / kWave);
  for (size_t kb = k0 + wave * kWave; kb < k1; kb += nwaves * kWave) {
    const size_t k = kb + lane;
    Vec16<T> cur;
    if (k < nfull) {
      cur = (NT & 1) ? load_nt(iv + k) : iv[k];
    } else {
#pragma unroll
      for (int j = 0; j < V; j++) {
        const size_t b = k * V + j;
        cur.v[j] = b < nbuf ? in[b] : T(0);
      }
    }
    // w[0..R): the R elements left of the vector, e[0..R): right of it
    T w[R], e[R];
#pragma unroll
    for (int d = 0; d < R; d++) {
      w[d] = wave_shift_up1(cur.v[V - R + d], T(0));
      e[d] = wave_shift_down1(cur.v[d], T(0));
    }
    if (lane == 0) {
#pragma unroll
      for (int d = 0; d < R; d++) {
        const size_t b = k * V - R + d; // wraps when k*V < R: then out of range
        w[d] = b < nbuf ? in[b] : T(0);
      }
    }
    if (lane == kWave - 1) {
#pragma unroll
      for (int d = 0; d < R; d++) {
        const size_t b = (k + 1) * V + d;
        e[d] = b < nbuf ? in[b] : T(0);
      }
    }
    if (k < k1) {
      C win[V + 2 * R];
#pragma unroll
      for (int d = 0; d < R; d++) {
        win[d] = (C)w[d];
        win[R + V + d] = (C)e[d];
      }
#pragma unroll
      for (int j = 0; j < V; j++) win[R + j] = (C)cur.v[j];
      Vec16<T> o;
      bool whole = true;
#pragma unroll
      for (int j = 0; j < V; j++) {
        C s = win[j];
#pragma unroll
        for (int d = 1; d <= 2 * R; d++) s += win[j + d];
        o.v[j] = (T)s;
        const size_t b = k * V + j;
        whole &= b >= lo_b && b < hi_b;
      }
      if (whole) {
        if (NT & 2)
          store_nt(ov + k, o);
        else
          ov[k] = o;
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

// Block-level form of stencil1d_vec: the loop is block-uniform, neighbours
// inside a wave come by DPP as there, and the R elements across a WAVE edge
// come through LDS from the neighbouring wave of the same block; only the
// two block edges load from global memory (2 per 1024-element block instead
// of 2 per 256-element wave), so nontemporal loads lose nothing at the wave
// edges.  NT bit 0 nontemporal loads, bit 1 nontemporal stores.
template <typename T, int R, int NT>
__global__ __launch_bounds__(kStThreads) void stencil1d_blk(const T *__restrict__ in, T *__restrict__ out,
                                                           size_t nbuf, size_t lo_b, size_t hi_b) {
  using C = typename ctype_of<T>::type;
  constexpr int V = Vec16<T>::N;
  constexpr int NW = kStThreads / kWave;
  static_assert(R <= V, "the neighbour vectors cover the radius");
  __shared__ T s_first[NW][R], s_last[NW][R];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const size_t nfull = nbuf / V;
  const size_t k0 = lo_b / V, k1 = (hi_b + V - 1) / V;
  const Vec16<T> *iv = reinterpret_cast<const Vec16<T> *>(in);
  Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out);
  for (size_t kb = k0 + (size_t)blockIdx.x * kStThreads; kb < k1; kb += (size_t)gridDim.x * kStThreads) {
    const size_t k = kb + tid;
    Vec16<T> cur;
    if (k < nfull) {
      cur = (NT & 1) ? load_nt(iv + k) : iv[k];
    } else {
#pragma unroll
      for (int j = 0; j < V; j++) {
        const size_t b = k * V + j;
        cur.v[j] = b < nbuf ? in[b] : T(0);
      }
    }
    T w[R], e[R];
#pragma unroll
    for (int d = 0; d < R; d++) {
      w[d] = wave_shift_up1(cur.v[V - R + d], T(0));
      e[d] = wave_shift_down1(cur.v[d], T(0));
    }
    if (lane == kWave - 1)
#pragma unroll
      for (int d = 0; d < R; d++) s_last[wid][d] = cur.v[V - R + d];
    if (lane == 0)
#pragma unroll
      for (int d = 0; d < R; d++) s_first[wid][d] = cur.v[d];
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int d = 0; d < R; d++) {
        if (wid > 0) {
          w[d] = s_last[wid - 1][d];
        } else {
          const size_t b = k * V - R + d; // wraps when k*V < R: then out of range
          w[d] = b < nbuf ? in[b] : T(0);
        }
      }
    }
    if (lane == kWave - 1) {
#pragma unroll
      for (int d = 0; d < R; d++) {
        if (wid < NW - 1) {
          e[d] = s_first[wid + 1][d];
        } else {
          const size_t b = (k + 1) * V + d;
          e[d] = b < nbuf ? in[b] : T(0);
        }
      }
    }
    __syncthreads(); // the next iteration rewrites s_first / s_last
    if (k < k1) {
      C win[V + 2 * R];
#pragma unroll
      for (int d = 0; d < R; d++) {
        win[d] = (C)w[d];
        win[R + V + d] = (C)e[d];
      }
#pragma unroll
      for (int j = 0; j < V; j++) win[R + j] = (C)cur.v[j];
      Vec16<T> o;
      bool whole = true;
#pragma unroll
      for (int j = 0; j < V; j++) {
        C sum = win[j];
#pragma unroll
        for (int d = 1; d <= 2 * R; d++) sum += win[j + d];
        o.v[j] = (T)sum;
        const size_t b = k * V + j;
        whole &= b >= lo_b && b < hi_b;
      }
      if (whole) {
        if (NT & 2)
          store_nt(ov + k, o);
        else
          ov[k] = o;
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

// Register-blocked 5-point 2-D stencil: one wave owns a strip of RB output
// rows x 64 column vectors.  It loads the strip's RB + 2 input rows once
// (RB + 2 independent 16-byte loads per lane in flight; interior rows
// nontemporal, the two halo rows shared with the neighbouring strips through
// L2) and produces RB output rows from registers, so each input vector is
// read ~(RB + 2) / RB times from L2 and once from HBM.  West/east neighbours
// come from DPP wave shifts; lanes 0 / 63 fetch the one element across the
// wave's column edge.  Strips are numbered row-block-major so the strips
// above and below one another run on the same XCD at about the same time.
#ifndef DRHIP_ST2D_RB
#define DRHIP_ST2D_RB 16
#endif
// cache policy (tools/stencil_nt.sh, 8192 x 65536 f32): bit 0 nontemporal
// interior-row loads, bit 1 nontemporal stores.  Nontemporal stores keep the
// output lines from evicting the input rows the neighbouring strips re-read
// from L2: 0.824 -> 0.735 ms (65 -> 73 % of HBM); nontemporal loads lose
// (0.93 ms).  The 1-D kernel keeps cached stores (0.732 vs 0.759 ms).
#ifndef DRHIP_ST2D_NT
#define DRHIP_ST2D_NT 2
#endif
// LDSE (DRHIP_ST2D_LDSE): when the block's waves are neighbouring column
// blocks of ONE row block (ncb a multiple of the waves per block), the
// column elements across a wave edge come from the neighbouring wave through
// LDS; only the block's two outer edges load them from global memory.
#ifndef DRHIP_ST2D_LDSE
#define DRHIP_ST2D_LDSE 1
#endif
template <typename T, int RB, int NT = DRHIP_ST2D_NT, bool LDSE = DRHIP_ST2D_LDSE>
__global__ __launch_bounds__(kStThreads) void stencil2d_strip(const T *__restrict__ in, T *__restrict__ out,
                                                             size_t nx, size_t rlo, size_t rhi, size_t ncb) {
  using C = typename ctype_of<T>::type;
  constexpr int V = Vec16<T>::N;
  constexpr int NW = kStThreads / kWave;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const size_t vpr = nx / V;
  const size_t item = ((size_t)blockIdx.x * kStThreads + threadIdx.x) / kWave;
  const size_t rb = item / ncb, cb = item - rb * ncb;
  const size_t r0 = rlo + rb * RB; // first output row (owned-row index)
  // block-uniform: every wave of the block in one row block
  const bool lds_edges = LDSE && ncb % NW == 0;
  if (r0 >= rhi) return; // wave-uniform (block-uniform when lds_edges)
  const int nr = (int)(rhi - r0 < (size_t)RB ? rhi - r0 : (size_t)RB);
  const size_t q = cb * kWave + lane; // column vector
  const bool act = q < vpr;
  // output row r0 + i - 1 (i = 1..nr) sits in buffer row r0 + i; the strip
  // reads buffer rows r0 .. r0 + nr + 1
  const Vec16<T> *iv = reinterpret_cast<const Vec16<T> *>(in) + r0 * vpr + q;
  Vec16<T> row[RB + 2];
#pragma unroll
  for (int i = 0; i < RB + 2; i++) {
    row[i] = Vec16<T>{};
    if (act && i <= nr + 1)
      row[i] = ((NT & 1) && i > 0 && i <= nr) ? load_nt(iv + (size_t)i * vpr) : iv[(size_t)i * vpr];
  }
  T wedge[RB], eedge[RB];
  const T *ie = in + r0 * nx + q * V;
  if (lds_edges) {
    __shared__ T s_w[NW][RB], s_e[NW][RB]; // a wave's first / last column element per row
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < RB; i++) s_w[wid][i] = row[i + 1].v[0];
    if (lane == kWave - 1)
#pragma unroll
      for (int i = 0; i < RB; i++) s_e[wid][i] = row[i + 1].v[V - 1];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RB; i++) {
      wedge[i] = T(0);
      eedge[i] = T(0);
      if (act && i < nr) {
        if (lane == 0 && q > 0) wedge[i] = wid > 0 ? s_e[wid - 1][i] : ie[(size_t)(i + 1) * nx - 1];
        if (lane == kWave - 1 && q + 1 < vpr) eedge[i] = wid < NW - 1 ? s_w[wid + 1][i] : ie[(size_t)(i + 1) * nx + V];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < RB; i++) {
      wedge[i] = T(0);
      eedge[i] = T(0);
      if (act && i < nr) {
        if (lane == 0 && q > 0) wedge[i] = ie[(size_t)(i + 1) * nx - 1];
        if (lane == kWave - 1 && q + 1 < vpr) eedge[i] = ie[(size_t)(i + 1) * nx + V];
      }
    }
  }
  Vec16<T> *ov = reinterpret_cast<Vec16<T> *>(out) + r0 * vpr + q;
  const bool inner = q != 0 && q != vpr - 1;
#pragma unroll
  for (int i = 1; i <= RB; i++) {
    const Vec16<T> &c = row[i];
    const T wv = wave_shift_up1(c.v[V - 1], wedge[i - 1]);
    const T ev = wave_shift_down1(c.v[0], eedge[i - 1]);
    Vec16<T> o;
#pragma unroll
    for (int j = 0; j < V; j++) {
      const C west = j == 0 ? (C)(lane == 0 ? wedge[i - 1] : wv) : (C)c.v[j - 1];
      const C east = j == V - 1 ? (C)(lane == kWave - 1 ? eedge[i - 1] : ev) : (C)c.v[j + 1];
      o.v[j] = (T)((C)c.v[j] + west + east + (C)row[i - 1].v[j] + (C)row[i + 1].v[j]);
    }
    if (act && i <= nr) {
      if (inner) {
        if (NT & 2)
          store_nt(ov + (size_t)i * vpr, o);
        else
          ov[(size_t)i * vpr] = o;
      } else {
        T *dst = reinterpret_cast<T *>(ov + (size_t)i * vpr);
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

// DRHIP_ST_NT (measurement): 1 nontemporal loads, 2 nontemporal stores, 3 both;
// unset = the shipped policy (cached 1-D, DRHIP_ST2D_NT for the 2-D strips)
static int stencil_nt() {
  const char *e = getenv("DRHIP_ST_NT");
  const int v = e ? atoi(e) : 0;
  return v >= 0 && v <= 3 ? v : 0;
}

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
      // one-shot grid (tools/copy_sweep.hip), grid-stride beyond 2^22 blocks
      unsigned grid = (unsigned)std::min<size_t>((nvec + kStThreads - 1) / kStThreads, size_t(1) << 22);
      const size_t nbuf = n_owned + 2 * (size_t)radius, lo_b = radius + lo, hi_b = radius + hi;
      // shipped: the block-level kernel (wave edges through LDS), cached
      // loads and stores (round 3: 0.693 vs 0.732 ms for the wave-level
      // kernel at 2^29 f32; nontemporal loads 0.76, stores 0.71-0.72,
      // both 0.74 -- tools/gpu_r03p.sh).  Measurement knobs:
      // DRHIP_ST1D_BLK=0 the wave-level stencil1d_vec, DRHIP_ST_NT the
      // cache policy of either (radius 1).
      const int nt = stencil_nt();
      const char *blk = getenv("DRHIP_ST1D_BLK");
      const bool wave_level = blk && atoi(blk) == 0;
      auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kStThreads), 0, s->stream, (const T *)in_buf, (T *)out_buf, nbuf,
                           lo_b, hi_b);
      };
      if (radius == 1 && nt) {
        if (wave_level) {
          if (nt == 1) launch(stencil1d_vec<T, 1, 1>);
          else if (nt == 2) launch(stencil1d_vec<T, 1, 2>);
          else launch(stencil1d_vec<T, 1, 3>);
        } else {
          if (nt == 1) launch(stencil1d_blk<T, 1, 1>);
          else if (nt == 2) launch(stencil1d_blk<T, 1, 2>);
          else launch(stencil1d_blk<T, 1, 3>);
        }
      } else if (wave_level) {
        if (radius == 1) launch(stencil1d_vec<T, 1>);
        else if (radius == 2) launch(stencil1d_vec<T, 2>);
        else if constexpr (V >= 4) {
          if (radius == 3) launch(stencil1d_vec<T, 3>);
          else launch(stencil1d_vec<T, 4>);
        }
      } else {
        if (radius == 1) launch(stencil1d_blk<T, 1, 0>);
        else if (radius == 2) launch(stencil1d_blk<T, 2, 0>);
        else if constexpr (V >= 4) {
          if (radius == 3) launch(stencil1d_blk<T, 3, 0>);
          else launch(stencil1d_blk<T, 4, 0>);
        }
      }
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
    static const bool rowvec = getenv("DRHIP_ST2D_ROWVEC") != nullptr; // measurement knob
    if (vec && !rowvec) {
      constexpr int RB = DRHIP_ST2D_RB;
      const size_t ncb = (nx / V + kWave - 1) / kWave;
      const size_t items = (rhi - rlo + RB - 1) / RB * ncb;
      const size_t grid = (items + kStThreads / kWave - 1) / (kStThreads / kWave);
      if (grid > 0x7fffffffu) return set_error(DRHIP_ERR_BAD_ARG, "drhip_stencil2d: grid too large");
      const int nt = stencil_nt();
#define DRHIP_ST2(NTV)                                                                                  \
  hipLaunchKernelGGL((stencil2d_strip<T, RB, NTV>), dim3((unsigned)grid), dim3(kStThreads), 0, s->stream, \
                     (const T *)in_buf, (T *)out_buf, nx, rlo, rhi, ncb)
      if (nt == 1) DRHIP_ST2(1);
      else if (nt == 2) DRHIP_ST2(2);
      else if (nt == 3) DRHIP_ST2(3);
      else DRHIP_ST2(DRHIP_ST2D_NT);
#undef DRHIP_ST2
    } else if (vec) {
      const size_t nvec = (rhi - rlo) * (nx / V);
      unsigned grid = (unsigned)std::min<size_t>((nvec + kStThreads - 1) / kStThreads, size_t(1) << 22);
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
