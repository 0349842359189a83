// pool_probe.hip -- does device memory from the stream-ordered pool
// (hipMallocAsync) read back what a kernel stored into it?  Round-1 saw stale
// D2H reads with a pool allocator (tools/dbg_fill.py); this isolates the
// allocation / kernel / copy / free stream placement of each step.
//
// Variants (each 36 fill + readback cases, as dbg_fill.py):
//   same     alloc, fill, free on the segment's non-blocking stream; blocking
//            hipMemcpy D2H into pageable memory after hipStreamSynchronize
//   pinned   same, D2H by hipMemcpyAsync on the stream into pinned memory
//   null     alloc / free on the NULL stream, fill on the non-blocking stream
//            (the allocation is not ordered before the fill)
//   keep     as `same`, pool release threshold = UINT64_MAX (memory kept)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));            \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

template <typename T> __global__ void fill_k(T *p, size_t n, T v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

template <typename T> static int run_case(const char *mode, hipStream_t s, size_t n, size_t off) {
  const size_t nb = (n + off) * sizeof(T);
  const bool null_alloc = !strcmp(mode, "null");
  T *p = nullptr;
  CK(hipMallocAsync((void **)&p, nb, null_alloc ? (hipStream_t)0 : s));
  unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(fill_k<T>, dim3(grid), dim3(256), 0, s, p + off, n, (T)7);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  std::vector<T> h(n + off);
  if (!strcmp(mode, "pinned")) {
    T *hp;
    CK(hipHostMalloc((void **)&hp, nb, 0));
    CK(hipMemcpyAsync(hp, p, nb, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    memcpy(h.data(), hp, nb);
    CK(hipHostFree(hp));
  } else {
    CK(hipMemcpy(h.data(), p, nb, hipMemcpyDeviceToHost));
  }
  size_t bad = 0;
  for (size_t i = off; i < n + off; i++) bad += h[i] != (T)7;
  CK(hipFreeAsync(p, null_alloc ? (hipStream_t)0 : s));
  return bad != 0;
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "same";
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (!strcmp(mode, "keep")) {
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    uint64_t thr = UINT64_MAX;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  }
  int tot = 0;
  const size_t cases[4][2] = {{4099, 0}, {100003, 3}, {100003, 0}, {1u << 20, 1}};
  for (int t = 0; t < 3; t++)
    for (auto &c : cases)
      for (int rep = 0; rep < 3; rep++) {
        if (t == 0) tot += run_case<int64_t>(mode, s, c[0], c[1]);
        if (t == 1) tot += run_case<int32_t>(mode, s, c[0], c[1]);
        if (t == 2) tot += run_case<double>(mode, s, c[0], c[1]);
      }
  CK(hipDeviceSynchronize());
  printf("pool_probe %s: failing cases %d of 36\n", mode, tot);
  CK(hipStreamDestroy(s));
  return 0;
}
