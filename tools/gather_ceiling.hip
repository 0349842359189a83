// gather_ceiling.hip -- measurement tool (not product): how many random
// 4-byte gathers per second an MI355X sustains, as a function of the gathers
// each lane keeps in flight (G), of the gathered table's size, and of
// whether the indices are computed (pure gathers) or streamed from memory
// (the CSR SpMV pattern: a 4-B colind load feeding each gather).
//
//   gather_hash<G>   lane issues G gathers at hashed indices (no index loads)
//   gather_idx<G>    lane loads G consecutive indices (G/4 16-B loads) from a
//                    streamed index array, then issues the G gathers
//   gather_spmv<G>   the random-C4 SpMV pattern: G indices AND G values per
//                    lane from two nontemporal 16-B streams (colind, vals),
//                    then the G gathers (round 4: does an x table small
//                    enough for the 256 MiB Infinity Cache -- 32 / 64 / 128
//                    MiB, i.e. a column panel of C4 -- gather faster while
//                    the 8 B-per-nonzero stream runs beside it?)
// Table sizes: 32 / 64 / 128 MiB (column panels), 256 MiB (C4's x: 2^26
// fp32) and 4 GiB (no cache reuse).
// Prints gathers/s per case; HBM 64-B-line model: 8e12 / 64 = 125 G lines/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int G>
__global__ __launch_bounds__(256) void gather_hash(const float *__restrict__ t, unsigned mask, size_t count,
                                                   float *out) {
  const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * G;
  if (i0 >= count) return;
  float v[G];
#pragma unroll
  for (int g = 0; g < G; g++) v[g] = t[hash32((unsigned)(i0 + g)) & mask];
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < G; g++) s += v[g];
  if (s == 12345.678f) out[0] = s;
}

template <int G>
__global__ __launch_bounds__(256) void gather_idx(const float *__restrict__ t, const unsigned *__restrict__ idx,
                                                  size_t count, float *out) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * G;
  if (i0 >= count) return;
  u4 ix[G / 4];
#pragma unroll
  for (int k = 0; k < G / 4; k++) ix[k] = *reinterpret_cast<const u4 *>(idx + i0 + 4 * k);
  float v[G];
#pragma unroll
  for (int k = 0; k < G / 4; k++) {
    v[4 * k + 0] = t[ix[k].x];
    v[4 * k + 1] = t[ix[k].y];
    v[4 * k + 2] = t[ix[k].z];
    v[4 * k + 3] = t[ix[k].w];
  }
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < G; g++) s += v[g];
  if (s == 12345.678f) out[0] = s;
}

template <int G>
__global__ __launch_bounds__(256) void gather_spmv(const float *__restrict__ t, const unsigned *__restrict__ idx,
                                                   const float *__restrict__ val, size_t count, float *out) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * G;
  if (i0 >= count) return;
  u4 ix[G / 4];
  f4 va[G / 4];
#pragma unroll
  for (int k = 0; k < G / 4; k++) {
    ix[k] = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(idx + i0 + 4 * k));
    va[k] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(val + i0 + 4 * k));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < G / 4; k++)
    s += va[k].x * t[ix[k].x] + va[k].y * t[ix[k].y] + va[k].z * t[ix[k].z] + va[k].w * t[ix[k].w];
  if (s == 12345.678f) out[0] = s;
}

__global__ void init_t(float *p, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = (float)(i & 0xFFFF) * (1.0f / 65536.0f);
}
__global__ void init_idx(unsigned *p, size_t n, unsigned mask) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = hash32((unsigned)i * 2654435761u + 12345u) & mask;
}

int main() {
  const size_t big = size_t(1) << 30;   // floats: 4 GiB table
  const size_t count = size_t(1) << 28; // gathers per launch
  float *t, *out, *val;
  unsigned *idx;
  CK(hipMalloc(&t, big * 4));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&idx, count * 4));
  CK(hipMalloc(&val, count * 4));
  hipLaunchKernelGGL(init_t, dim3((unsigned)(count / 256)), dim3(256), 0, 0, val, count);
  hipLaunchKernelGGL(init_t, dim3((unsigned)(big / 256)), dim3(256), 0, 0, t, big);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float m = 0;
      CK(hipEventElapsedTime(&m, e0, e1));
      ms.push_back(m);
    }
    float best = ms[0];
    for (float m : ms) best = m < best ? m : best;
    return best;
  };
  const bool panels = getenv("GATHER_PANELS") != nullptr;
  for (unsigned log2t : panels ? std::vector<unsigned>{23u, 24u, 25u, 26u, 30u} : std::vector<unsigned>{26u, 30u}) {
    const unsigned mask = (1u << log2t) - 1u;
    hipLaunchKernelGGL(init_idx, dim3((unsigned)(count / 256)), dim3(256), 0, 0, idx, count, mask);
    CK(hipDeviceSynchronize());
    auto run = [&](const char *name, int g, auto launch) {
      const float ms = timeit(launch);
      printf("{\"kernel\": \"%s\", \"G\": %d, \"table_MiB\": %zu, \"ms\": %.4f, \"Ggathers_per_s\": %.2f}\n", name, g,
             (size_t(4) << log2t) >> 20, ms, count / (ms * 1e-3) / 1e9);
      fflush(stdout);
    };
#define RUN_G(G)                                                                                                \
  run("hash", G, [&] {                                                                                          \
    hipLaunchKernelGGL(gather_hash<G>, dim3((unsigned)(count / G / 256)), dim3(256), 0, 0, t, mask, count, out); \
  });                                                                                                           \
  run("idx", G, [&] {                                                                                           \
    hipLaunchKernelGGL(gather_idx<G>, dim3((unsigned)(count / G / 256)), dim3(256), 0, 0, t, idx, count, out);   \
  });
    if (panels) {
      // the SpMV pattern at every table size, and the plain index gathers
      run("spmv", 8, [&] {
        hipLaunchKernelGGL(gather_spmv<8>, dim3((unsigned)(count / 8 / 256)), dim3(256), 0, 0, t, idx, val, count, out);
      });
      run("spmv", 16, [&] {
        hipLaunchKernelGGL(gather_spmv<16>, dim3((unsigned)(count / 16 / 256)), dim3(256), 0, 0, t, idx, val, count,
                           out);
      });
      run("idx", 8, [&] {
        hipLaunchKernelGGL(gather_idx<8>, dim3((unsigned)(count / 8 / 256)), dim3(256), 0, 0, t, idx, count, out);
      });
      continue;
    }
    run("hash", 1, [&] {
      hipLaunchKernelGGL(gather_hash<1>, dim3((unsigned)(count / 256)), dim3(256), 0, 0, t, mask, count, out);
    });
    RUN_G(4)
    RUN_G(8)
    RUN_G(16)
    RUN_G(32)
  }
  CK(hipFree(t));
  CK(hipFree(out));
  CK(hipFree(idx));
  CK(hipFree(val));
  return 0;
}
