// stencil_sweep.hip -- measurement tool (not product): shapes of the 3-point
// fp32 1-D stencil (out[i] = in[i-1] + in[i] + in[i+1]) on 2^29 cells, to
// find why the product kernel trails the one-shot copy ceiling
// (tools/copy_sweep.hip).  Every variant is checked against variant 0.
// Build: make -C tools stencil_sweep.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float shr1(float x, float fill) { // lane i <- lane i-1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, fill),
                                                               __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float shl1(float x, float fill) { // lane i <- lane i+1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, fill),
                                                               __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, false));
}

// buffer in[0..n+2): owned cells 1..n; out[i] for i in [1, n+1)
// variant 0: plain scalar, one cell per thread (reference shape)
__global__ __launch_bounds__(256) void v0(const float *in, float *out, size_t n) {
  size_t i = 1 + blockIdx.x * (size_t)256 + threadIdx.x;
  if (i <= n) out[i] = in[i - 1] + in[i] + in[i + 1];
}

// vector k covers cells [4k, 4k+4); out written for cells in [1, n+1)
template <int EDGE, bool NT, bool NTS = NT>
__global__ __launch_bounds__(256) void vdpp(const float *in, float *out, size_t n) {
  const size_t nv = (n + 2) / 4; // full vectors of the buffer (n+2 multiple of 4 here)
  const size_t k = blockIdx.x * (size_t)256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  f4 c = k < nv ? (NT ? __builtin_nontemporal_load((const f4 *)in + k) : ((const f4 *)in)[k]) : f4{0, 0, 0, 0};
  float wl = 0, er = 0;
  if (EDGE == 0) { // edge lanes load the whole neighbouring vector
    if (lane == 0 && k > 0) wl = ((const f4 *)in)[k - 1].w;
    if (lane == 63 && k + 1 < nv) er = ((const f4 *)in)[k + 1].x;
  } else if (EDGE == 1) { // edge lanes load one element
    if (lane == 0 && k > 0) wl = in[4 * k - 1];
    if (lane == 63 && k + 1 < nv) er = in[4 * k + 4];
  } else { // every lane loads its two neighbour elements (no DPP)
    if (k > 0 && k < nv) wl = in[4 * k - 1];
    if (k + 1 < nv) er = in[4 * k + 4];
  }
  float w = EDGE == 2 ? wl : shr1(c.w, wl);
  float e = EDGE == 2 ? er : shl1(c.x, er);
  if (EDGE != 2) {
    if (lane == 0) w = wl;
    if (lane == 63) e = er;
  }
  f4 o;
  o.x = w + c.x + c.y;
  o.y = c.x + c.y + c.z;
  o.z = c.y + c.z + c.w;
  o.w = c.z + c.w + e;
  if (k < nv) {
    if (k > 0 && k + 1 < nv) {
      if (NTS)
        __builtin_nontemporal_store(o, (f4 *)out + k);
      else
        ((f4 *)out)[k] = o;
    } else {
      for (int j = 0; j < 4; j++) {
        size_t b = 4 * k + j;
        if (b >= 1 && b <= n) out[b] = o[j];
      }
    }
  }
}

// LDS staging: block stages its 256 vectors (+ one element each side)
__global__ __launch_bounds__(256) void vlds(const float *in, float *out, size_t n) {
  __shared__ float s[1024 + 2];
  const size_t nv = (n + 2) / 4;
  const size_t k0 = blockIdx.x * (size_t)256, k = k0 + threadIdx.x;
  f4 c = k < nv ? __builtin_nontemporal_load((const f4 *)in + k) : f4{0, 0, 0, 0};
  *(f4 *)&s[1 + 4 * threadIdx.x] = c; // unaligned-by-one LDS store (4 dwords)
  if (threadIdx.x == 0) s[0] = k0 > 0 ? in[4 * k0 - 1] : 0.f;
  if (threadIdx.x == 255) s[1025] = 4 * (k0 + 256) < n + 2 ? in[4 * (k0 + 256)] : 0.f;
  __syncthreads();
  const float *p = &s[1 + 4 * threadIdx.x];
  f4 o;
  o.x = p[-1] + p[0] + p[1];
  o.y = p[0] + p[1] + p[2];
  o.z = p[1] + p[2] + p[3];
  o.w = p[2] + p[3] + p[4];
  if (k < nv) {
    if (k > 0 && k + 1 < nv) {
      __builtin_nontemporal_store(o, (f4 *)out + k);
    } else {
      for (int j = 0; j < 4; j++) {
        size_t b = 4 * k + j;
        if (b >= 1 && b <= n) out[b] = o[j];
      }
    }
  }
}

__global__ void fill(float *x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = (float)((i * 2654435761u) >> 8 & 0xFFFF) / 65536.0f;
}

static const size_t N = (size_t(1) << 29) - 2; // owned cells; buffer = 2^29

template <typename F> double timeit(F f, hipStream_t st) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float tot = 0;
  const int reps = 10;
  for (int r = -2; r < reps; r++) {
    CK(hipEventRecord(e0, st));
    f();
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 0) tot += ms;
  }
  return tot / reps;
}

int main() {
  const size_t nb = N + 2;
  float *in, *out, *ref;
  CK(hipMalloc(&in, nb * 4));
  CK(hipMalloc(&out, nb * 4));
  CK(hipMalloc(&ref, nb * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, in, nb);
  CK(hipMemsetAsync(ref, 0, nb * 4, st));
  const unsigned g1 = (unsigned)((N + 255) / 256), gv = (unsigned)((nb / 4 + 255) / 256);
  double ms = timeit([&] { hipLaunchKernelGGL(v0, dim3(g1), dim3(256), 0, st, in, ref, N); }, st);
  printf("%-28s %7.3f ms %7.1f GB/s\n", "scalar one cell/thread", ms, 8.0 * N / ms / 1e6);
  std::vector<float> h(nb), hr(nb);
  CK(hipMemcpy(hr.data(), ref, nb * 4, hipMemcpyDeviceToHost));
  auto check = [&](const char *name, double ms) {
    CK(hipMemcpy(h.data(), out, nb * 4, hipMemcpyDeviceToHost));
    bool ok = memcmp(h.data() + 1, hr.data() + 1, N * 4) == 0;
    printf("%-28s %7.3f ms %7.1f GB/s %s\n", name, ms, 8.0 * N / ms / 1e6, ok ? "ok" : "MISMATCH");
  };
#define RUNV(K, name)                                                                          \
  CK(hipMemsetAsync(out, 0, nb * 4, st));                                                      \
  ms = timeit([&] { hipLaunchKernelGGL(K, dim3(gv), dim3(256), 0, st, in, out, N); }, st); \
  check(name, ms);
  RUNV((vdpp<0, true>), "dpp, edge vector, nt");
  RUNV((vdpp<1, true>), "dpp, edge element, nt");
  RUNV((vdpp<2, true>), "per-lane neighbour loads, nt");
  RUNV((vdpp<1, false>), "dpp, edge element");
  RUNV(vlds, "lds staged, nt");
  RUNV((vdpp<1, false, true>), "dpp, edge element, nts");
  RUNV((vdpp<0, false, true>), "dpp, edge vector, nts");
  RUNV((vdpp<0, false, false>), "dpp, edge vector");
  return 0;
}
