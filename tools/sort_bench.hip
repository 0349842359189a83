// sort_bench.hip -- measurement tool (not product): times drhip_sort (via the
// C-ABI) on n uint32 keys and, as a yardstick only, rocPRIM's radix sort on
// the same keys.  Build: make -C tools sort_bench.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/drhip.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define CD(x)                                                                      \
  do {                                                                             \
    int r_ = (x);                                                                  \
    if (r_) {                                                                      \
      fprintf(stderr, "%s:%d drhip %d %s\n", __FILE__, __LINE__, r_, drhip_last_error()); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void gen(uint32_t *x, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    x[i] = (uint32_t)h;
  }
}

int main(int argc, char **argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 28;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const size_t n = size_t(1) << log2n;
  int dev = 0;
  CD(drhip_init(&dev, 1));
  hipStream_t st;
  CD(drhip_stream(0, (void **)&st));
  uint32_t *keys, *src;
  CK(hipMalloc(&keys, n * 4));
  CK(hipMalloc(&src, n * 4));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, st, src, n, 12345u);
  size_t wsb = 0;
  CD(drhip_sort_workspace(0, DRHIP_U32, n, &wsb));
  void *ws;
  CK(hipMalloc(&ws, wsb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float tot = 0;
  for (int r = -1; r < reps; r++) {
    CK(hipMemcpyAsync(keys, src, n * 4, hipMemcpyDeviceToDevice, st));
    CK(hipEventRecord(e0, st));
    CD(drhip_sort(0, DRHIP_U32, keys, n, ws, wsb));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 0) tot += ms;
  }
  const double ms = tot / reps;
  // check sortedness + checksum equality on a sample
  std::vector<uint32_t> h(n), hs(n);
  CK(hipMemcpy(h.data(), keys, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hs.data(), src, n * 4, hipMemcpyDeviceToHost));
  bool sorted = std::is_sorted(h.begin(), h.end());
  uint64_t s1 = 0, s2 = 0;
  for (size_t i = 0; i < n; i++) {
    s1 += h[i];
    s2 += hs[i];
  }
  printf("drhip_sort  u32 n=2^%d  %8.3f ms  %7.2f Gkeys/s  algorithmic 48 B/key -> %7.1f GB/s  sorted=%d sum_ok=%d\n",
         log2n, ms, n / ms / 1e6, 48.0 * n / ms / 1e6, (int)sorted, (int)(s1 == s2));
  // rocPRIM yardstick
  uint32_t *out;
  CK(hipMalloc(&out, n * 4));
  size_t tb = 0;
  CK(rocprim::radix_sort_keys(nullptr, tb, src, out, n, 0, 32, st));
  void *tmp;
  CK(hipMalloc(&tmp, tb));
  tot = 0;
  for (int r = -1; r < reps; r++) {
    CK(hipEventRecord(e0, st));
    CK(rocprim::radix_sort_keys(tmp, tb, src, out, n, 0, 32, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float m;
    CK(hipEventElapsedTime(&m, e0, e1));
    if (r >= 0) tot += m;
  }
  printf("rocprim     u32 n=2^%d  %8.3f ms  %7.2f Gkeys/s (yardstick only)\n", log2n, tot / reps, n / (tot / reps) / 1e6);
  CD(drhip_finalize());
  return 0;
}
